// Which workgroups share a CU? 512 workgroups of 256 threads with 80 KB of LDS each (two per
// CU); each records HW_ID (CU / SH / SE) and XCC_ID plus its start time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned* out, int spin) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x * 2] = hw;
    out[blockIdx.x * 2 + 1] = xcc;
    lds[0] = 1;
  }
  for (int k = 0; k < spin; ++k) __builtin_amdgcn_s_sleep(127);
}

int main() {
  const int nb = 1024;
  unsigned* d;
  hipMalloc(&d, nb * 2 * 4);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 80 * 1024, 0, d, 64);
  hipDeviceSynchronize();
  std::vector<unsigned> h(nb * 2);
  hipMemcpy(h.data(), d, nb * 2 * 4, hipMemcpyDeviceToHost);
  std::map<unsigned, std::vector<int>> cu;
  for (int b = 0; b < nb; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const unsigned key = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
    cu[key].push_back(b);
  }
  printf("%zu distinct CUs\n", cu.size());
  int shown = 0;
  for (auto& kv : cu) {
    if (shown++ < 24) {
      printf("xcc %u se %u sh %u cu %2u:", kv.first >> 16, (kv.first >> 8) & 7, (kv.first >> 4) & 1, kv.first & 0xf);
      for (int b : kv.second) printf(" %d", b);
      printf("\n");
    }
  }
  return 0;
}
