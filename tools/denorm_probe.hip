#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(float* out, float v) {
  const int lane = threadIdx.x;
  f16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)0.0f; b[e] = (_Float16)0.0f; }
  // single product: A[0][0] * B[0][0]
  if (lane == 0) { a[0] = (_Float16)v; b[0] = (_Float16)1.0f; }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  if (lane == 0) { out[0] = acc[0]; out[1] = (float)(_Float16)v; }
}
int main() {
  float* d; hipMalloc(&d, 8);
  float vs[3] = {1e-3f, 1e-5f, 1e-7f};
  for (float v : vs) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, v);
    float h[2]; hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("v=%g  cvt=%g  mfma=%g\n", v, h[1], h[0]);
  }
  return 0;
}
