#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));
__global__ void probe(const float* a, const float* b, float* out) {
  const int l = threadIdx.x;
  floatx16 c;
  for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_f32_16x16x1f32(a[l], b[l], c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) out[i * 64 + l] = c[i];
}
int main() {
  float ha[64], hb[64], ho[1024];
  float *da, *db, *dout;
  hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dout, 4096);
  for (int pass = 0; pass < 2; ++pass) {
    for (int l = 0; l < 64; ++l) { ha[l] = pass == 0 ? l : 1.f; hb[l] = pass == 0 ? 1.f : l; }
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice); hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dout);
    hipMemcpy(ho, dout, 4096, hipMemcpyDeviceToHost);
    printf("pass %d (%s lane supplying the %s)\n", pass, pass == 0 ? "A" : "B", pass == 0 ? "row" : "col");
    for (int i = 0; i < 16; ++i) {
      printf("v%02d:", i);
      for (int l = 0; l < 64; ++l) printf(" %2d", (int)ho[i * 64 + l]);
      printf("\n");
    }
  }
  return 0;
}
