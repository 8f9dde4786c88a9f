// f64 MFMA probe (gfx950): operand / result lane maps of v_mfma_f64_4x4x4_4b_f64
// and issue costs beside v_fma_f64.  Diagnostic only; not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// wave w: A lane l = 1000 + l, B one-hot at lane w -> D (64 x 64 table)
__global__ void map_kernel(double* out, int which) {
  const int l = threadIdx.x & 63, w = blockIdx.x;
  double a, b;
  if (which == 0) { a = 1000.0 + l; b = (l == w) ? 1.0 : 0.0; }   // probe B lanes
  else            { b = 1000.0 + l; a = (l == w) ? 1.0 : 0.0; }   // probe A lanes
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[w * 64 + l] = d;
}

// timing: N iterations of U independent accumulators
template <int U, int MODE>
__global__ void time_kernel(const double* in, double* out, long long* cyc, int n) {
  const int l = threadIdx.x & 63;
  double a = in[l], b = in[64 + l];
  double acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = in[128 + u];
  double f[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) f[u] = in[200 + u];
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE != 2) acc[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[u], 0, 0, 0);
      if (MODE >= 1) {
#pragma unroll
        for (int v = 0; v < 8; ++v) f[v] = fma(f[v], a, b);
      }
    }
  }
  long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += acc[u];
#pragma unroll
  for (int u = 0; u < 8; ++u) s += f[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int U, int MODE>
void run_time(const char* name, int waves_per_simd) {
  double *in, *out; long long* cyc;
  CK(hipMalloc(&in, 4096 * 8)); CK(hipMalloc(&out, 1 << 20)); CK(hipMalloc(&cyc, 4096 * 8));
  double h[4096]; for (int i = 0; i < 4096; ++i) h[i] = 1e-3 * (i % 17);
  CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
  const int n = 2000;
  // one workgroup of 4*waves_per_simd waves per CU... use 1 WG on one CU
  hipLaunchKernelGGL((time_kernel<U, MODE>), dim3(1), dim3(64 * 4 * waves_per_simd), 0, 0, in, out, cyc, n);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((time_kernel<U, MODE>), dim3(1), dim3(64 * 4 * waves_per_simd), 0, 0, in, out, cyc, n);
  CK(hipDeviceSynchronize());
  long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  // clock64 = s_memtime (shader clock ticks)
  printf("%-28s wps=%d U=%d: %.2f cycles per inner iteration per wave (%lld total)\n", name, waves_per_simd, U,
         (double)c / (n * U), c);
  CK(hipFree(in)); CK(hipFree(out)); CK(hipFree(cyc));
}

int main() {
  double* out; CK(hipMalloc(&out, 64 * 64 * 8));
  double h[64 * 64];
  for (int which = 0; which < 2; ++which) {
    hipLaunchKernelGGL(map_kernel, dim3(64), dim3(64), 0, 0, out, which);
    CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    printf("MAP %s\n", which == 0 ? "B" : "A");
    for (int w = 0; w < 64; ++w) {
      printf("%d:", w);
      for (int l = 0; l < 64; ++l) if (h[w * 64 + l] != 0.0) printf(" %d=%g", l, h[w * 64 + l]);
      printf("\n");
    }
  }
  run_time<1, 0>("mfma dependent", 1);
  run_time<4, 0>("mfma 4 indep", 1);
  run_time<8, 0>("mfma 8 indep", 1);
  run_time<4, 2>("8 fma per slot (no mfma)", 1);
  run_time<4, 1>("mfma + 8 fma", 1);
  run_time<4, 0>("mfma 4 indep", 2);
  run_time<4, 2>("8 fma per slot (no mfma)", 2);
  run_time<4, 1>("mfma + 8 fma", 2);
  return 0;
}
