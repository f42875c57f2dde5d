// Can the f32 VALU add throughput beside f32 MFMA on gfx950?  Each workgroup holds
// `mw` MFMA waves (v_mfma_f32_32x32x2_f32 loop, operands in registers) and `vw` VALU waves
// (v_pk_fma_f32 loop, 16 independent float2 chains).  Prints the combined f32 rate, so
// MFMA-only, VALU-only and mixed runs can be compared at the same launch shape: if the two
// pipes run side by side under the chip's power limit, a GEMM could hand part of its tile
// to VALU waves.
//
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/hybrid_ceiling tools/hybrid_ceiling.hip
// usage: hybrid_ceiling [n_wg] [mfma_waves] [valu_waves] [mfma_per_wave] [pkfma_per_wave] [warmup]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(1024, 1) void k_hybrid(const float* seed, float* out, int mw, int mfma_iters,
                                                    int valu_iters) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  const int wave = threadIdx.x >> 6;
  float s = 0.f;
  if (wave < mw) {
    float a0 = seed[t & 1023], a1 = seed[(t + 7) & 1023], b0 = seed[(t + 13) & 1023], b1 = seed[(t + 29) & 1023];
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    for (int it = 0; it < mfma_iters; ++it) {
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[i][e];
  } else {
    f32x2 a = {seed[t & 1023], seed[(t + 3) & 1023]};
    f32x2 b = {seed[(t + 5) & 1023], seed[(t + 11) & 1023]};
    f32x2 c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = f32x2{seed[(t + i) & 1023], 0.f};
    for (int it = 0; it < valu_iters; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = __builtin_elementwise_fma(a, b, c[i]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c[i][0] + c[i][1];
  }
  out[t] = s;
}

int main(int argc, char** argv) {
  const int nwg = argc > 1 ? atoi(argv[1]) : 256;
  const int mw = argc > 2 ? atoi(argv[2]) : 4;
  const int vw = argc > 3 ? atoi(argv[3]) : 4;
  const long mfma = argc > 4 ? atol(argv[4]) : 64000;
  const long pk = argc > 5 ? atol(argv[5]) : 128000;
  const int warm = argc > 6 ? atoi(argv[6]) : 20;
  const int mfma_iters = (int)(mfma / 4), valu_iters = (int)(pk / 16);
  float h[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) h[i] = (float)rand() / RAND_MAX - 0.5f;
  float *seed, *out;
  hipMalloc(&seed, sizeof(h));
  hipMalloc(&out, (size_t)nwg * (mw + vw) * 64 * sizeof(float));
  hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 blk((mw + vw) * 64);
  for (int w = 0; w < warm; ++w) hipLaunchKernelGGL(k_hybrid, dim3(nwg), blk, 0, 0, seed, out, mw, mfma_iters, valu_iters);
  const int reps = 10;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_hybrid, dim3(nwg), blk, 0, 0, seed, out, mw, mfma_iters, valu_iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double sec = ms * 1e-3 / reps;
  const double fm = 2.0 * 32 * 32 * 2 * (double)mfma_iters * 4 * nwg * mw;
  const double fv = 2.0 * 2 * 64 * (double)valu_iters * 16 * nwg * vw;
  printf("wg %d: %d mfma waves x %ld mfma, %d valu waves x %ld pk_fma: %.1f us/launch, mfma %.1f + valu %.1f = %.1f TFLOP/s\n",
         nwg, mw, mfma, vw, pk, sec * 1e6, fm / sec / 1e12, fv / sec / 1e12, (fm + fv) / sec / 1e12);
  return 0;
}
