// Copy floor of one 4096^2 x 2 FP64 plane pair (268 MB read + 268 MB written,
// the algorithmic bytes of one stencil pass): which streaming-copy shape reaches
// the guide's ~6.3 TB/s?  Variants: grid-stride vs one-shot unrolled, 16 B per
// lane, plain / non-temporal stores, grid sizes, waves per workgroup.
//
//   hipcc --offload-arch=gfx950 -O3 -o copy_floor copy_floor.hip && ./copy_floor
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void st(d2v *p, d2v v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride, one 16-B element per lane per iteration
template <bool NT>
__global__ __launch_bounds__(256) void copy_gs(const d2v *__restrict__ s, d2v *__restrict__ d, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) st<NT>(d + i, s[i]);
}

// one-shot: each workgroup copies a contiguous block of U * 256 elements, U loads in flight per lane
template <bool NT, int U, int BS>
__global__ __launch_bounds__(BS) void copy_os(const d2v *__restrict__ s, d2v *__restrict__ d, long n) {
    const long base = (long)blockIdx.x * U * BS + threadIdx.x;
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * BS;
        v[u] = i < n ? s[i] : d2v{0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * BS;
        if (i < n) st<NT>(d + i, v[u]);
    }
}

template <typename F>
static float time_us(F launch, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 5; ++w) launch(w);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / reps;
}

int main() {
    const long n_cells = 2L * 4096 * 4096;
    const long bytes = n_cells * 8;
    const long n = n_cells / 2;
    d2v *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 0, bytes);
    (void)hipMemset(b, 0, bytes);
    const double alg = 2.0 * bytes;
    auto report = [&](const char *name, float us) {
        printf("{\"kernel\": \"%s\", \"us\": %.1f, \"alg_TBps\": %.3f, \"frac_8TBps\": %.3f}\n", name, us,
               alg / (us * 1e-6) / 1e12, alg / (us * 1e-6) / 8e12);
    };
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        char nm[64];
        snprintf(nm, sizeof nm, "grid_stride_nt_g%d", g);
        report(nm, time_us([&](int r) { hipLaunchKernelGGL(copy_gs<true>, dim3(g), dim3(256), 0, 0, (r & 1) ? b : a, (r & 1) ? a : b, n); }, 20));
        snprintf(nm, sizeof nm, "grid_stride_plain_g%d", g);
        report(nm, time_us([&](int r) { hipLaunchKernelGGL(copy_gs<false>, dim3(g), dim3(256), 0, 0, (r & 1) ? b : a, (r & 1) ? a : b, n); }, 20));
    }
#define OS(NT, U, BS)                                                                                              \
    {                                                                                                              \
        const long per = (long)(U) * (BS);                                                                         \
        report("oneshot_" #NT "_U" #U "_B" #BS, time_us([&](int r) {                                               \
                   hipLaunchKernelGGL((copy_os<NT, U, BS>), dim3((n + per - 1) / per), dim3(BS), 0, 0,              \
                                      (r & 1) ? b : a, (r & 1) ? a : b, n);                                         \
               }, 20));                                                                                            \
    }
    OS(true, 1, 256) OS(true, 2, 256) OS(true, 4, 256) OS(true, 8, 256) OS(true, 16, 256)
    OS(false, 1, 256) OS(false, 4, 256) OS(false, 8, 256)
    OS(true, 4, 64) OS(true, 8, 64) OS(true, 4, 512) OS(true, 4, 1024)
    return 0;
}
