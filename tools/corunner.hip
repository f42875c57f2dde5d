// Co-runner kernels for isolating a cross-workgroup interference seen on gfx950 (see
// DESIGN.md §5): while another process checks a kernel for run-to-run determinism, this
// one loops a single instruction pattern on every CU for ~12 s.
//   mode 0: v_mfma_f32_32x32x16_f16 register loop (no LDS)
//   mode 1: v_mfma_f32_32x32x2_f32 register loop (no LDS)
//   mode 2: LDS traffic only (ds_write_b64 + ds_read_b128 of f16x8), 56 KB allocated
//   mode 3: mode 0's MFMA loop with 56 KB of LDS allocated (unused)
//   mode 4: v_mfma_f32_16x16x32_f16 register loop (no LDS)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/corunner tools/corunner.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_run(const float* seed, float* out, int iters, int mode) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  float s = 0.f;
  if (mode == 0 || mode == 3) {
    f16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)seed[(t + i) & 1023]; b[i] = (_Float16)seed[(t + 3 * i) & 1023]; }
    f32x16 acc[2] = {};
    for (int it = 0; it < iters; ++it) {
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[1], 0, 0, 0);
    }
    for (int e = 0; e < 16; ++e) s += acc[0][e] + acc[1][e];
  } else if (mode == 1) {
    float a = seed[t & 1023], b = seed[(t + 5) & 1023];
    f32x16 acc[2] = {};
    for (int it = 0; it < iters; ++it) {
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc[1], 0, 0, 0);
    }
    for (int e = 0; e < 16; ++e) s += acc[0][e] + acc[1][e];
  } else if (mode == 4) {
    f16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)seed[(t + i) & 1023]; b[i] = (_Float16)seed[(t + 3 * i) & 1023]; }
    f32x4 acc[2] = {};
    for (int it = 0; it < iters; ++it) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc[1], 0, 0, 0);
    }
    for (int e = 0; e < 4; ++e) s += acc[0][e] + acc[1][e];
  } else {  // mode 2: LDS only, inside the 56 KB allocation
    const int n = 28 * 1024;  // uint16 elements
    for (int it = 0; it < iters / 8; ++it) {
      const int w = ((threadIdx.x * 4 + it * 64) & (n / 4 - 1)) * 4;
      u32x2 v = {(uint32_t)it, (uint32_t)t};
      *reinterpret_cast<u32x2*>(sm + w) = v;
      __syncthreads();
      const f16x8 r = *reinterpret_cast<const f16x8*>(sm + ((threadIdx.x * 8 + it * 8) & (n - 8)));
      s += (float)r[0];
      __syncthreads();
    }
  }
  out[t] = s;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const double secs = argc > 2 ? atof(argv[2]) : 12.0;
  float h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (float)((i * 37) % 101) / 101.f - 0.5f;
  float *seed, *out;
  const int nwg = 1024;
  hipMalloc(&seed, sizeof(h));
  hipMalloc(&out, (size_t)nwg * 256 * sizeof(float));
  hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
  const size_t lds = (mode == 2 || mode == 3) ? 56 * 1024 : 0;
  auto t0 = std::chrono::steady_clock::now();
  long n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_run, dim3(nwg), dim3(256), lds, 0, seed, out, 2048, mode);
    hipDeviceSynchronize();
    ++n;
  }
  printf("corunner mode %d done %ld\n", mode, n);
  return 0;
}
