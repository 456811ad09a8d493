#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double v4d __attribute__((ext_vector_type(4)));
// A 16x4, B 4x16 row-major; C 16x16 row-major
__global__ void k(const double* A, const double* B, double* C, int* map) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];   // A[i=l&15][k=l>>4]
  double b = B[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][j=l&15]
  v4d c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r, col = l & 15;
    C[row * 16 + col] = c[r];
  }
}
int main() {
  double hA[64], hB[64], hC[256], ref[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 7) % 13 - 6; hB[i] = (i * 5) % 11 - 5; }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int kk = 0; kk < 4; ++kk) s += hA[i*4+kk]*hB[kk*16+j]; ref[i*16+j] = s; }
  double *dA, *dB, *dC; int* dm;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 2048); hipMalloc(&dm, 4);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipMemset(dC, 0, 2048);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dm);
  hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 256; ++i) if (hC[i] != ref[i]) ++bad;
  printf("mfma_f64_16x16x4 layout check: %d mismatches of 256\n", bad);
  return bad != 0;
}
