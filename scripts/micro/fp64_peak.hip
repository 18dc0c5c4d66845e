// FP64 VALU throughput probe: independent fma / add chains, and DPP movs.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int MODE>
__global__ __launch_bounds__(256) void k(double *out, int iters, double a, double b) {
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3 + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (MODE == 0) x[j] = fma(x[j], a, b);
            else if (MODE == 1) x[j] = x[j] + b;
            else {
                int2 v = __builtin_bit_cast(int2, x[j]);
                v.x = __builtin_amdgcn_mov_dpp(v.x, 0x138, 0xf, 0xf, true);
                v.y = __builtin_amdgcn_mov_dpp(v.y, 0x138, 0xf, 0xf, true);
                x[j] = __builtin_bit_cast(double, v) + b;
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    int blocks = 256 * 8 * 4, iters = 4096;
    double *out;
    hipMalloc(&out, (size_t)blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999, 1e-3);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999, 1e-3);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999, 1e-3);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            double ops = (double)blocks * 256 * iters * 8;   // lane-instructions (f64 op)
            if (rep == 2) printf("mode %d (%s): %.3f ms, %.2f T lane-op/s (x2 for fma flops)\n", mode,
                                 mode == 0 ? "fma" : mode == 1 ? "add" : "2dpp+add", ms, ops / ms / 1e9);
        }
    }
    return 0;
}
