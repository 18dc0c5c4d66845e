// Streaming copy bandwidth (16 B per lane, grid-stride) by working-set size:
// does a plane pair that fits the 256 MiB Infinity Cache stream faster than HBM?
// Reports read+write GB/s for plain and non-temporal stores, back-to-back reps.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <bool NT>
__global__ __launch_bounds__(256) void copy(const double2 *__restrict__ s, double2 *__restrict__ d, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        double2 v = s[i];
        if (NT) {
            typedef double d2v __attribute__((ext_vector_type(2)));
            d2v w = {v.x, v.y};
            __builtin_nontemporal_store(w, reinterpret_cast<d2v *>(d + i));
        } else {
            d[i] = v;
        }
    }
}

template <bool NT>
static void run(double2 *a, double2 *b, long bytes) {
    const long n = bytes / 16;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int grid = 256 * 16;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(copy<NT>, dim3(grid), dim3(256), 0, 0, a, b, n);
    const int reps = 20;
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) {
        // ping-pong like the stencil passes: a -> b, b -> a
        if (r & 1) hipLaunchKernelGGL(copy<NT>, dim3(grid), dim3(256), 0, 0, b, a, n);
        else hipLaunchKernelGGL(copy<NT>, dim3(grid), dim3(256), 0, 0, a, b, n);
    }
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%s stores, %6.1f MB per buffer (%6.1f MB moved per copy): %7.1f GB/s, %7.2f us per copy\n",
           NT ? "nt   " : "plain", bytes / 1e6, 2 * bytes / 1e6, 2.0 * bytes * reps / (ms * 1e-3) / 1e9,
           ms * 1e3 / reps);
}

int main() {
    const long max_bytes = 1L << 30;
    double2 *a, *b;
    (void)hipMalloc(&a, max_bytes);
    (void)hipMalloc(&b, max_bytes);
    (void)hipMemset(a, 0, max_bytes);
    (void)hipMemset(b, 0, max_bytes);
    for (long mb : {16L, 32L, 64L, 96L, 128L, 192L, 268L, 512L, 1024L}) {
        long bytes = mb << 20;
        if (mb == 268) bytes = 268435456L;   // one 4096^2 x 2-plane set
        run<false>(a, b, bytes);
        run<true>(a, b, bytes);
    }
    return 0;
}
