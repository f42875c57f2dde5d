// Accuracy of cos candidates for the RFF epilogue on gfx950 (tools/cos_accuracy.hip):
//   lib  = OCML cosf (the shipped epilogue),
//   hw   = v_cos_f32 (__builtin_amdgcn_cosf, input in revolutions) after a Cody-Waite reduction
//          of z to r in [-pi, pi] (k = rint(z / 2pi), three-part 2pi),
//   hwn  = v_cos_f32 on z / 2pi directly (no reduction),
// against cos((double) z), over z uniform in [-R, R] for R in {4, 64, 512, 4096}.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/cos_accuracy tools/cos_accuracy.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ inline float u01(uint32_t x) {  // hash -> [0, 1)
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (x >> 8) * (1.0f / 16777216.0f);
}

__global__ void k_err(float R, int n, unsigned long long* out) {
  // out[0..2]: max abs error (as double bits, non-negative so integer max works) of lib, hw, hwn
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float z = (2.f * u01((uint32_t)i * 2654435761u + 12345u) - 1.f) * R;
  const double ref = cos((double)z);
  const float lib = cosf(z);
  const float k = __builtin_rintf(z * 0.15915494309189535f);
  float r = __builtin_fmaf(-k, 6.28318548202514648f, z);
  r = __builtin_fmaf(-k, -1.7484555314695172e-7f, r);
  r = __builtin_fmaf(-k, -2.3889859e-15f, r);
  const float hw = __builtin_amdgcn_cosf(r * 0.15915494309189535f);
  const float hwn = __builtin_amdgcn_cosf(z * 0.15915494309189535f);
  const double e[3] = {fabs((double)lib - ref), fabs((double)hw - ref), fabs((double)hwn - ref)};
  for (int j = 0; j < 3; ++j) atomicMax(out + j, (unsigned long long)__double_as_longlong(e[j]));
}

int main() {
  const int n = 1 << 24;
  unsigned long long* d;
  hipMalloc(&d, 3 * sizeof(unsigned long long));
  for (float R : {4.f, 64.f, 512.f, 4096.f}) {
    hipMemset(d, 0, 3 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_err, dim3(n / 256), dim3(256), 0, 0, R, n, d);
    unsigned long long h[3];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double e[3];
    for (int j = 0; j < 3; ++j) memcpy(&e[j], &h[j], 8);
    printf("|z| <= %6.0f: max |err| vs cos(double z): OCML cosf %.3e, v_cos after Cody-Waite %.3e, v_cos direct %.3e\n",
           R, e[0], e[1], e[2]);
  }
  hipFree(d);
  return 0;
}
