// Probe: accuracy of gfx950 native sin/cos (v_sin_f32 / v_cos_f32, input in
// revolutions) and OCML sincospif against double, over phase fractions [0,1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const double* f, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = (float)f[i];
  out[6*i+0] = __builtin_amdgcn_sinf(x);
  out[6*i+1] = __builtin_amdgcn_cosf(x);
  float s, c; sincospif(2.0f * x, &s, &c);
  out[6*i+2] = s; out[6*i+3] = c;
  out[6*i+4] = __sinf(6.283185307179586f * x);
  out[6*i+5] = __cosf(6.283185307179586f * x);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> f(n);
  for (int i = 0; i < n; i++) f[i] = (double)(float)((i + 0.37) / n);
  double* df; float* dout;
  hipMalloc(&df, n * 8); hipMalloc(&dout, n * 24);
  hipMemcpy(df, f.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(df, dout, n);
  std::vector<float> o(6 * n);
  hipMemcpy(o.data(), dout, n * 24, hipMemcpyDeviceToHost);
  double e[3] = {0, 0, 0};
  for (int i = 0; i < n; i++) {
    double s = sin(2 * M_PI * f[i]), c = cos(2 * M_PI * f[i]);
    for (int m = 0; m < 3; m++) {
      e[m] = fmax(e[m], fabs(o[6*i+2*m] - s));
      e[m] = fmax(e[m], fabs(o[6*i+2*m+1] - c));
    }
  }
  printf("max abs err: native_rev %.3e  sincospif %.3e  __sinf %.3e\n", e[0], e[1], e[2]);
  return 0;
}
