// Self-test of the gfx950 cross-lane idioms and the f64 MFMA layout that
// chol_mfma_kernel relies on (exact integer data; asymmetric B).
//   hipcc --offload-arch=gfx950 -O2 -o lane_ops_test lane_ops_test.hip && ./lane_ops_test
// Prints "LANE_OPS_OK" and exits 0 when every check passes.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int G>
__device__ double bcast_group(double x) {
  unsigned lo = __double2loint(x), hi = __double2hiint(x);
  auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  unsigned l2 = (G < 2) ? a[0] : a[1], h2 = (G < 2) ? b[0] : b[1];
  auto c = __builtin_amdgcn_permlane16_swap(l2, l2, false, false);
  auto d = __builtin_amdgcn_permlane16_swap(h2, h2, false, false);
  unsigned l3 = (G & 1) ? c[1] : c[0], h3 = (G & 1) ? d[1] : d[0];
  return __hiloint2double((int)h3, (int)l3);
}

__global__ void k_bcast(double* out) {
  const int l = threadIdx.x;
  const double x = 1000.0 + l;
  out[0 * 64 + l] = bcast_group<0>(x);
  out[1 * 64 + l] = bcast_group<1>(x);
  out[2 * 64 + l] = bcast_group<2>(x);
  out[3 * 64 + l] = bcast_group<3>(x);
}

// D = A*B with A[i][k] = i*4+k+1, B[k][j] = 100*k + j + 7 (asymmetric)
__global__ void k_mfma(double* out) {
  const int l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  const double a = i * 4 + kk + 1, b = 100.0 * kk + i + 7;   // lane l: A[l&15][l>>4], B[l>>4][l&15]
  v4d acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];   // C/D: row (l>>4)+4r, col l&15
}

// f64 MFMA with BLGP = 1: negate A (CDNA f64 MFMA reuses BLGP as neg flags)
__global__ void k_mfma_neg(double* out) {
  const int l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  const double a = i * 4 + kk + 1, b = 100.0 * kk + i + 7;
  v4d acc = {1, 2, 3, 4};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 1);
  for (int r = 0; r < 4; ++r) out[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

int main() {
  double *d, h[256];
  if (hipMalloc(&d, 256 * sizeof(double)) != hipSuccess) return 2;
  int bad = 0;
  hipLaunchKernelGGL(k_bcast, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 256 * sizeof(double), hipMemcpyDeviceToHost);
  for (int g = 0; g < 4; ++g)
    for (int l = 0; l < 64; ++l)
      if (h[g * 64 + l] != 1000.0 + 16 * g + (l & 15)) {
        if (bad++ < 8) printf("bcast<%d> lane %d: %g\n", g, l, h[g * 64 + l]);
      }
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 256 * sizeof(double), hipMemcpyDeviceToHost);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double want = 0;
      for (int k = 0; k < 4; ++k) want += (i * 4 + k + 1) * (100.0 * k + j + 7);
      if (h[i * 16 + j] != want) {
        if (bad++ < 16) printf("mfma D[%d][%d] = %g want %g\n", i, j, h[i * 16 + j], want);
      }
    }
  hipLaunchKernelGGL(k_mfma_neg, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 256 * sizeof(double), hipMemcpyDeviceToHost);
  int negbad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double want = 0;
      for (int k = 0; k < 4; ++k) want += (i * 4 + k + 1) * (100.0 * k + j + 7);
      const double init = 1.0 + ((i >> 2) & 3);   // acc[r] = r + 1 for row (l>>4) + 4r
      if (h[i * 16 + j] != init - want) negbad++;
    }
  printf(negbad ? "BLGP1_NEGATES_A: no (%d mismatches)\n" : "BLGP1_NEGATES_A: yes\n", negbad);
  hipFree(d);
  if (bad) { printf("LANE_OPS_FAIL %d\n", bad); return 1; }
  printf("LANE_OPS_OK\n");
  return 0;
}
