// Which XCDs / CUs a CU-masked stream's workgroups land on (ON THE GPU BOX):
//   hipcc --offload-arch=gfx950 -O2 -o tools/cumask_probe tools/cumask_probe.hip && tools/cumask_probe
// For masks of CU-number groups (8 consecutive numbers; several layouts), a kernel of 4096
// workgroups records each workgroup's XCC_ID and HW_ID (s_getreg, read only); the host counts the
// distinct XCDs and (XCD, SE, CU) triples used.  Tells whether HIP deals CU numbers to the XCDs in
// turn or in contiguous ranges.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void where(uint32_t *out) {
  if (threadIdx.x == 0) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // keep the workgroup resident for a while so the grid spreads over every CU the mask allows
  const uint64_t t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < 200000) {
  }
}

int main() {
  int n = 0;
  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", n);
  const int nwg = 4096;
  uint32_t *d;
  hipMalloc(&d, nwg * 2 * sizeof(uint32_t));
  std::vector<uint32_t> h(nwg * 2);
  struct Case { const char *name; std::vector<int> groups; };  // groups of 8 CU numbers
  std::vector<Case> cases = {{"all", {}}, {"group 0 (CUs 0-7)", {0}}, {"groups 0-3 (CUs 0-31)", {0, 1, 2, 3}},
                             {"groups 24-31 (CUs 192-255)", {24, 25, 26, 27, 28, 29, 30, 31}},
                             {"every 4th group (3, 7, ..., 31)", {3, 7, 11, 15, 19, 23, 27, 31}}};
  for (auto &c : cases) {
    std::vector<uint32_t> mask((n + 31) / 32, c.groups.empty() ? 0xFFFFFFFFu : 0u);
    for (int g : c.groups)
      for (int i = 8 * g; i < 8 * g + 8 && i < n; ++i) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
      printf("%s: stream create failed\n", c.name);
      continue;
    }
    hipMemsetAsync(d, 0xFF, nwg * 2 * sizeof(uint32_t), s);
    hipLaunchKernelGGL(where, dim3(nwg), dim3(64), 0, s, d);
    hipMemcpyAsync(h.data(), d, nwg * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    std::set<uint32_t> xcds;
    std::set<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>> cus;
    std::vector<int> per_xcd(16, 0);
    for (int i = 0; i < nwg; ++i) {
      const uint32_t x = h[2 * i] & 15u, hw = h[2 * i + 1];
      xcds.insert(x);
      per_xcd[x]++;
      // HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
      cus.insert({x, (hw >> 13) & 7u, (hw >> 12) & 1u, (hw >> 8) & 15u});
    }
    printf("%-34s XCDs used %zu, distinct (xcd, se, sh, cu) %zu; workgroups per XCD:", c.name, xcds.size(), cus.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per_xcd[x]);
    printf("\n");
    hipStreamDestroy(s);
  }
  hipFree(d);
  return 0;
}
