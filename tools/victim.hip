// Victim kernels for the cross-process interference seen on gfx950: each mode
// computes a deterministic result; the reference is taken before the co-runner starts (the
// program sleeps 4 s after it), then the kernel is re-run for ~6 s and every result is
// compared bit for bit; mismatching lanes are reported by their lane index within the wave.
//   mode 0: per-thread f32 fma chain (VALU only)
//   mode 1: the same chain with the x operand read from LDS (16 threads broadcast one row)
//   mode 2: tanhf of an fma chain
//   mode 3: f64 sin/cos/log (Box-Muller)
//   mode 4: mode 1 with the weight rows read from LDS too (the policy kernel's pattern)
//   mode 5: mode 1 with every lane reading its own LDS row (no broadcast)
//   mode 6: mode 1 with the broadcast row read as 4 x ds_read_b32
// build: hipcc --offload-arch=gfx950 -O3 -o tools/victim tools/victim.hip
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_victim(const float* in, float* out, int mode) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int t = threadIdx.x, g = blockIdx.x * 256 + t;
  const int l = t / 16, u = t % 16;
  float r = 0.f;
  if (mode == 0 || mode == 2) {
    float acc = 0.f;
    for (int k = 0; k < 200; ++k) acc = fmaf(in[(g * 7 + k) & 4095], in[(k * 13 + u) & 4095], acc);
    r = mode == 2 ? tanhf(acc) : acc;
  } else if (mode == 3) {
    const double u1 = 1.0 - (double)((g * 2654435761u) & 0xffffff) / 16777216.0;
    const double u2 = (double)((g * 40503u) & 0xffff) / 65536.0;
    r = (float)(sqrt(-2.0 * log(u1)) * (u & 1 ? sin(6.283185307179586 * u2) : cos(6.283185307179586 * u2)));
  } else if (mode == 5 || mode == 6) {
    float* xs = lds;  // [256][52] for mode 5 (own row), [16][204] for mode 6
    const int rows = mode == 5 ? 256 : 16, ld = mode == 5 ? 52 : 204;
    for (int i = t; i < rows * ld; i += 256) xs[i] = in[(blockIdx.x * 16 * 204 + i) & 4095];
    __syncthreads();
    float acc0 = 0.f;
    const float* row = xs + (mode == 5 ? t : l) * ld;
    if (mode == 5) {
      for (int k = 0; k < 12; ++k) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(row + 4 * k);
        const float a0 = in[(u * 4 + k) & 4095];
        acc0 = fmaf(a0, v.x, acc0); acc0 = fmaf(a0, v.y, acc0); acc0 = fmaf(a0, v.z, acc0); acc0 = fmaf(a0, v.w, acc0);
      }
    } else {
      for (int k = 0; k < 200; ++k) acc0 = fmaf(in[(u * 4 + k) & 4095], row[(k * 37) % 200], acc0);
    }
    r = acc0;
  } else {  // 1, 4: rows of x in LDS (16 lanes x 200), weights (32 x 204) in LDS for mode 4
    float* xs = lds;                 // [16][204]
    float* ws = lds + 16 * 204;      // [32][204]
    for (int i = t; i < 16 * 204; i += 256) xs[i] = in[(blockIdx.x * 16 * 204 + i) & 4095];
    for (int i = t; i < 32 * 204; i += 256) ws[i] = in[(i * 3 + 1) & 4095];
    __syncthreads();
    float acc0 = 0.f, acc1 = 0.f;
    for (int k = 0; k < 50; ++k) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xs + l * 204 + 4 * k);
      f32x4 a0, a1;
      if (mode == 4) {
        a0 = *reinterpret_cast<const f32x4*>(ws + u * 204 + 4 * k);
        a1 = *reinterpret_cast<const f32x4*>(ws + (u + 16) * 204 + 4 * k);
      } else {
        a0 = f32x4{in[(u * 4 + k) & 4095], in[(u * 4 + k + 1) & 4095], in[(u * 4 + k + 2) & 4095], in[(u * 4 + k + 3) & 4095]};
        a1 = a0 * 0.5f;
      }
      acc0 = fmaf(a0.x, v.x, acc0); acc0 = fmaf(a0.y, v.y, acc0); acc0 = fmaf(a0.z, v.z, acc0); acc0 = fmaf(a0.w, v.w, acc0);
      acc1 = fmaf(a1.x, v.x, acc1); acc1 = fmaf(a1.y, v.y, acc1); acc1 = fmaf(a1.z, v.z, acc1); acc1 = fmaf(a1.w, v.w, acc1);
    }
    r = acc0 + acc1;
  }
  out[g] = r;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int nwg = 64, n = nwg * 256;
  std::vector<float> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 37) % 101) / 101.f - 0.5f;
  float *in, *out;
  hipMalloc(&in, 4096 * sizeof(float));
  hipMalloc(&out, n * sizeof(float));
  hipMemcpy(in, h.data(), 4096 * sizeof(float), hipMemcpyHostToDevice);
  const size_t lds = (mode == 1 || mode == 4) ? 48 * 204 * 4 : (mode == 5 ? 256 * 52 * 4 : (mode == 6 ? 16 * 204 * 4 : 0));
  std::vector<float> ref(n), cur(n);
  hipLaunchKernelGGL(k_victim, dim3(nwg), dim3(256), lds, 0, in, out, mode);
  hipMemcpy(ref.data(), out, n * sizeof(float), hipMemcpyDeviceToHost);
  sleep(4);
  long runs = 0, bad = 0;
  int lanebad[64] = {0};
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 6.0) {
    hipLaunchKernelGGL(k_victim, dim3(nwg), dim3(256), lds, 0, in, out, mode);
    hipMemcpy(cur.data(), out, n * sizeof(float), hipMemcpyDeviceToHost);
    ++runs;
    bool any = false;
    for (int i = 0; i < n; ++i)
      if (memcmp(&cur[i], &ref[i], 4)) { any = true; lanebad[i & 63]++; }
    bad += any;
  }
  printf("victim mode %d: %ld of %ld runs differ; wave lanes:", mode, bad, runs);
  for (int i = 0; i < 64; ++i) if (lanebad[i]) printf(" %d", i);
  printf("\n");
  return 0;
}
