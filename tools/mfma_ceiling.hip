// MFMA-only ceiling of v_mfma_f32_32x32x2_f32 on this chip, at the ensemble GEMM's grid:
// each wave runs the same number of MFMAs as one 128x128 (or 256x128) output tile of the
// K = 1769 hidden layer, operands in registers (no LDS, no global traffic), random data.
// Tells how much of the gap between the GEMM and the 157.3 TF spec is clock (DVFS under
// f32 MFMA load) rather than the kernel's schedule.
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_ceiling tools/mfma_ceiling.hip
// usage: mfma_ceiling [n_wg] [waves_per_wg] [mfma_per_wave] [zero_operands] [warmup_launches]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512, 1) void k_ceiling(const float* seed, float* out, int iters) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  float a0 = seed[t & 1023], a1 = seed[(t + 7) & 1023], b0 = seed[(t + 13) & 1023], b1 = seed[(t + 29) & 1023];
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[i][e];
  out[t] = s;
}

int main(int argc, char** argv) {
  const int nwg = argc > 1 ? atoi(argv[1]) : 512;
  const int wpw = argc > 2 ? atoi(argv[2]) : 8;
  const long mfma = argc > 3 ? atol(argv[3]) : 3584;  // 128x128 tile, K=1792: 4 tiles x 896 steps / wave
  const int zero = argc > 4 ? atoi(argv[4]) : 0;
  const int warm = argc > 5 ? atoi(argv[5]) : 3;
  const int iters = (int)(mfma / 4);
  float h[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) h[i] = zero ? 0.f : (float)rand() / RAND_MAX - 0.5f;
  float *seed, *out;
  hipMalloc(&seed, sizeof(h));
  hipMalloc(&out, (size_t)nwg * wpw * 64 * sizeof(float));
  hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < warm; ++w) hipLaunchKernelGGL(k_ceiling, dim3(nwg), dim3(wpw * 64), 0, 0, seed, out, iters);
  const int reps = 20;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_ceiling, dim3(nwg), dim3(wpw * 64), 0, 0, seed, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * (double)iters * 4 * nwg * wpw;
  printf("wg %d x %d waves, %ld mfma/wave, %s operands, %d warmup: %.1f us/launch, %.1f TFLOP/s\n", nwg, wpw,
         mfma, zero ? "zero" : "random", warm, ms * 1e3 / reps, flops * reps / (ms * 1e-3) / 1e12);
  return 0;
}
