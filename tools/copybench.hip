// copybench.hip — measurement tool (not product): device-to-device copy variants, to find the
// box's HBM copy ceiling (bench.py's copy16 measured 4.9-5.1 TB/s against the guide's
// 6.29 TB/s float4 copy).  Rate = (bytes read + bytes written) / time, as bench.py reports it.
//   copybench [GiB]          prints one line per variant: name  TB/s (best of 5 after a warm-up)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// grid-stride, U 16-byte loads in flight per thread, then U stores; NTL/NTS: non-temporal loads/stores
template <int U, bool NTL, bool NTS, int T>
__global__ __launch_bounds__(T) void copy_gs(const u32x4 *src, u32x4 *dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * T * U;
  for (uint64_t i = (uint64_t)blockIdx.x * T * U + threadIdx.x; i < n16; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + (uint64_t)u * T;
      const u32x4 *p = src + (j < n16 ? j : i);
      v[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + (uint64_t)u * T;
      if (j < n16) {
        if (NTS) __builtin_nontemporal_store(v[u], dst + j);
        else dst[j] = v[u];
      }
    }
  }
}

// one pass: every thread copies U consecutive-by-T elements once (grid covers the buffer)
template <int U, bool NTL, bool NTS, int T>
__global__ __launch_bounds__(T) void copy_flat(const u32x4 *src, u32x4 *dst, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * T * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t j = i + (uint64_t)u * T;
    const u32x4 *p = src + (j < n16 ? j : 0);
    v[u] = NTL ? __builtin_nontemporal_load(p) : *p;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t j = i + (uint64_t)u * T;
    if (j < n16) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + j);
      else dst[j] = v[u];
    }
  }
}

static int g_cus = 256;

template <class K>
static void run(const char *name, K kern, unsigned grid, unsigned threads, const u32x4 *s, u32x4 *d, uint64_t n16) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, s, d, n16);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, s, d, n16);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  printf("%-40s grid %7u  %.3f ms  %.3f TB/s\n", name, grid, best, 2.0 * n16 * 16 / (best * 1e-3) / 1e12);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

#define GS(U, L, S, T, MULT)                                                                              \
  run("gs U=" #U " ntl=" #L " nts=" #S " T=" #T " x" #MULT, copy_gs<U, L, S, T>, (unsigned)(g_cus * MULT), T, \
      src, dst, n16)
#define FLAT(U, L, S, T)                                                                                  \
  run("flat U=" #U " ntl=" #L " nts=" #S " T=" #T, copy_flat<U, L, S, T>,                                 \
      (unsigned)((n16 + (uint64_t)T * U - 1) / ((uint64_t)T * U)), T, src, dst, n16)

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  const uint64_t n16 = bytes / 16;
  int dev = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
  u32x4 *src, *dst;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipMemset(dst, 0, bytes));
  printf("copy of %.2f GiB, %d CUs\n", gib, g_cus);
  GS(4, true, true, 256, 8);  // the product copy16 before round 4
  GS(4, true, true, 256, 16);
  GS(4, true, true, 256, 32);
  GS(8, true, true, 256, 8);
  GS(8, true, true, 256, 16);
  GS(2, true, true, 256, 16);
  GS(4, false, false, 256, 8);
  GS(4, false, false, 256, 16);
  GS(4, false, true, 256, 16);
  GS(4, true, false, 256, 16);
  GS(8, false, false, 256, 16);
  GS(4, true, true, 512, 8);
  GS(4, true, true, 1024, 4);
  GS(1, false, false, 256, 32);
  FLAT(1, false, false, 256);
  FLAT(2, false, false, 256);
  FLAT(4, false, false, 256);
  FLAT(4, true, true, 256);
  FLAT(8, true, true, 256);
  FLAT(4, false, true, 256);
  FLAT(1, true, true, 256);
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
