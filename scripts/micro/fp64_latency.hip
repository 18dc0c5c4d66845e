// FP64 VALU issue rate vs independent chains per wave (CH) and waves per SIMD (W):
// how much ILP / TLP a wave64 f64 add stream needs to saturate the SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CH>
__global__ __launch_bounds__(256) void k(double *out, int iters, double b) {
    double x[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) x[j] = threadIdx.x * 1e-3 + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16 / CH; ++r) {
#pragma unroll
            for (int j = 0; j < CH; ++j) x[j] = x[j] + b;
        }
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) s += x[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
static void run(double *out, int w) {
    const int blocks = 256 * w, iters = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double ops = (double)blocks * 256 * iters * 16;
    printf("chains %d waves/SIMD %d: %.2f T lane-add/s\n", CH, w, ops / best / 1e9);
}

int main() {
    double *out;
    (void)hipMalloc(&out, (size_t)256 * 16 * 256 * 8);
    for (int w = 1; w <= 4; ++w) {
        run<1>(out, w);
        run<2>(out, w);
        run<4>(out, w);
        run<8>(out, w);
    }
    return 0;
}
