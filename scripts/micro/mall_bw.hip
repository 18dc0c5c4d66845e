// Streaming bandwidth against the working-set size: does a pass whose source and
// destination fit the 256 MiB Infinity Cache (MALL) stream faster than HBM?
// Copies ping-pong A -> B -> A over buffer pairs of 8 MiB .. 512 MiB each, one
// 16-B element per thread (the copy-floor shape of copy_floor.hip), with plain
// (cached) or non-temporal stores, plus a read-only reduction.
//
//   hipcc --offload-arch=gfx950 -O3 -o mall_bw mall_bw.hip && ./mall_bw
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ __launch_bounds__(256) void copy1(const d2v *__restrict__ s, d2v *__restrict__ d, long n) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i < n) {
        if (NT) __builtin_nontemporal_store(s[i], d + i);
        else d[i] = s[i];
    }
}

// read-only: 4 elements per thread, one 8-B partial per block written (negligible)
__global__ __launch_bounds__(256) void read4(const d2v *__restrict__ s, double *out, long n) {
    const long base = blockIdx.x * 1024L + threadIdx.x;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long i = base + u * 256L;
        if (i < n) { const d2v v = s[i]; acc += v.x + v.y; }
    }
    if (acc == 12345.678) out[blockIdx.x] = acc;   // never true for the zero buffers: keeps the loads
}

template <typename F>
static float time_us(F launch, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 6; ++w) launch(w);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / reps;
}

int main() {
    const long max_bytes = 512L << 20;
    d2v *a, *b;
    double *out;
    if (hipMalloc(&a, max_bytes) != hipSuccess || hipMalloc(&b, max_bytes) != hipSuccess ||
        hipMalloc(&out, 1 << 22) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, max_bytes);
    (void)hipMemset(b, 0, max_bytes);
    for (long mib : {8L, 16L, 32L, 48L, 64L, 96L, 128L, 160L, 192L, 256L, 384L, 512L}) {
        const long bytes = mib << 20, n = bytes / 16;
        const unsigned g = (unsigned)((n + 255) / 256), g4 = (unsigned)((n + 1023) / 1024);
        const int reps = mib <= 64 ? 200 : 40;
        const float t_plain = time_us([&](int r) {
            hipLaunchKernelGGL(copy1<false>, dim3(g), dim3(256), 0, 0, (r & 1) ? b : a, (r & 1) ? a : b, n); }, reps);
        const float t_nt = time_us([&](int r) {
            hipLaunchKernelGGL(copy1<true>, dim3(g), dim3(256), 0, 0, (r & 1) ? b : a, (r & 1) ? a : b, n); }, reps);
        const float t_rd = time_us([&](int r) {
            hipLaunchKernelGGL(read4, dim3(g4), dim3(256), 0, 0, (r & 1) ? b : a, out, n); }, reps);
        printf("{\"mib_per_buffer\": %ld, \"copy_plain_us\": %.2f, \"copy_plain_TBps\": %.2f, \"copy_nt_us\": %.2f, "
               "\"copy_nt_TBps\": %.2f, \"read_us\": %.2f, \"read_TBps\": %.2f}\n",
               mib, t_plain, 2.0 * bytes / (t_plain * 1e-6) / 1e12, t_nt, 2.0 * bytes / (t_nt * 1e-6) / 1e12, t_rd,
               (double)bytes / (t_rd * 1e-6) / 1e12);
        fflush(stdout);
    }
    return 0;
}
