// Cost of switching between kernels with and without > 64 KB of LDS per workgroup (gfx950 has
// 160 KB of LDS per CU).  Sequences of 8 launches of the same streaming-write kernel, each with
// `lds` bytes of dynamic LDS: all 0, all 80 KB, alternating, and 0/32 KB / 32 KB/80 KB.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_switch.hip -o tools/bin/lds_switch
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_write(float4* p, long n, float v) {
    extern __shared__ float lds[];
    if (threadIdx.x == 1023) lds[0] = v;  // never true: keeps the LDS request
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = make_float4(v, v + 1, v + 2, v + 3);
}

int main() {
    float4* p;
    CK(hipMalloc(&p, 64 << 20));
    CK(hipFuncSetAttribute((const void*)k_write, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int cases[][2] = {{0, 0}, {80, 80}, {0, 80}, {0, 32}, {32, 80}, {64, 65}, {0, 64}, {0, 65}};
    for (int mb : {1, 16}) {
        const long n = ((long)mb << 20) / 16;
        for (int rep = 0; rep < 2; ++rep)
            for (auto& c : cases) {
                float best = 1e9f;
                for (int it = 0; it < 20; ++it) {
                    CK(hipEventRecord(e0));
                    for (int k = 0; k < 8; ++k)
                        k_write<<<1024, 256, (k & 1 ? c[1] : c[0]) * 1024>>>(p, n, it);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms < best ? ms : best;
                }
                if (rep) printf("%2d MB x 8 launches, LDS %2d KB / %2d KB alternating: %8.2f us\n", mb, c[0], c[1], best * 1e3f);
            }
    }
    return 0;
}
