// Memory floor of the stencil pass's access pattern: the wave-tile geometry of
// variant 6 (128-column tiles of which 128 - 2*KH are written, ROWS output rows
// per tile, rows [c0-K-2, c1+K) read at 16 B per lane, 6 rows prefetched,
// streaming stores) with the arithmetic removed, against a plain streaming copy
// of the same two planes.  The gap between the stencil pass and this kernel is
// what the arithmetic costs; the gap between this kernel and the copy is what
// the tile halos and the tile-shaped access pattern cost.
//
//   hipcc --offload-arch=gfx950 -O3 -o stencil_mem stencil_mem.hip && ./stencil_mem [n]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d2v __attribute__((ext_vector_type(2)));

template <int K, int ROWS, int COLS_PER_LANE>
__global__ __launch_bounds__(256) void tile_copy(const double *__restrict__ src, double *dst, long fstride, int ny,
                                                 int nx, int tiles_x, int chunks_y, int nf) {
    constexpr int KH = K + (K & 1);
    constexpr int WT = 64 * COLS_PER_LANE;
    constexpr int W = WT - 2 * KH;
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (wave >= tiles_x * chunks_y * nf) return;
    const int tx = wave % tiles_x, ty = (wave / tiles_x) % chunks_y, f = wave / (tiles_x * chunks_y);
    const int c0 = ty * ROWS, c1 = min(c0 + ROWS, nx);
    int cA = tx * W - KH + COLS_PER_LANE * lane;
    cA = min(max(cA, 0), ny - COLS_PER_LANE);
    const bool w = lane >= KH / COLS_PER_LANE && lane < 64 - KH / COLS_PER_LANE;
    const double *s = src + f * fstride;
    double *d = dst + f * fstride;
    d2v pf[6][COLS_PER_LANE / 2];
    const int i0 = c0 - K - 2, i1 = c1 + K;
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
        for (int h = 0; h < COLS_PER_LANE / 2; ++h)
            pf[u][h] = *reinterpret_cast<const d2v *>(s + (long)min(max(i0 + u, 0), nx - 1) * ny + cA + 2 * h);
    for (int i = i0; i < i1; i += 6) {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            d2v v[COLS_PER_LANE / 2];
#pragma unroll
            for (int h = 0; h < COLS_PER_LANE / 2; ++h) {
                v[h] = pf[u][h];
                pf[u][h] = *reinterpret_cast<const d2v *>(s + (long)min(max(i + u + 6, 0), nx - 1) * ny + cA + 2 * h);
            }
            const int r = i + u - K;
            if (r >= c0 && r < c1 && w)
#pragma unroll
                for (int h = 0; h < COLS_PER_LANE / 2; ++h)
                    __builtin_nontemporal_store(v[h], reinterpret_cast<d2v *>(d + (long)r * ny + cA + 2 * h));
        }
    }
}

__global__ __launch_bounds__(256) void copy(const d2v *__restrict__ s, d2v *__restrict__ d, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        __builtin_nontemporal_store(s[i], d + i);
}

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) launch(w);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(r);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

template <int K, int ROWS, int CPL>
static void run_tile(double *a, double *b, long fstride, int n) {
    constexpr int KH = K + (K & 1);
    constexpr int W = 64 * CPL - 2 * KH;
    const int tiles_x = (n + W - 1) / W, chunks_y = (n + ROWS - 1) / ROWS, nf = 2;
    const int waves = tiles_x * chunks_y * nf;
    const float ms = time_ms([&](int r) {
        hipLaunchKernelGGL((tile_copy<K, ROWS, CPL>), dim3((waves + 3) / 4), dim3(256), 0, 0, (r & 1) ? b : a,
                           (r & 1) ? a : b, fstride, n, n, tiles_x, chunks_y, nf);
    }, 20);
    const double alg = 16.0 * 2 * (double)n * n;   // one 8-B read + one 8-B write per cell
    printf("{\"kernel\": \"tile_copy\", \"K\": %d, \"rows\": %d, \"cols_per_lane\": %d, \"waves\": %d, \"us\": %.1f, "
           "\"alg_GBps\": %.0f}\n", K, ROWS, CPL, waves, ms * 1e3, alg / (ms * 1e-3) / 1e9);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const long fstride = (long)n * n;
    double *a, *b;
    if (hipMalloc(&a, 2 * fstride * 8) != hipSuccess || hipMalloc(&b, 2 * fstride * 8) != hipSuccess) return 1;
    (void)hipMemset(a, 0, 2 * fstride * 8);
    (void)hipMemset(b, 0, 2 * fstride * 8);
    const long nv = 2 * fstride / 2;
    const float ms = time_ms([&](int r) {
        hipLaunchKernelGGL(copy, dim3(256 * 16), dim3(256), 0, 0, (const d2v *)((r & 1) ? b : a),
                           (d2v *)((r & 1) ? a : b), nv);
    }, 20);
    printf("{\"kernel\": \"copy\", \"us\": %.1f, \"alg_GBps\": %.0f}\n", ms * 1e3,
           16.0 * 2 * (double)n * n / (ms * 1e-3) / 1e9);
    run_tile<9, 64, 2>(a, b, fstride, n);
    run_tile<9, 32, 2>(a, b, fstride, n);
    run_tile<9, 128, 2>(a, b, fstride, n);
    run_tile<9, 256, 2>(a, b, fstride, n);
    run_tile<9, 64, 4>(a, b, fstride, n);
    run_tile<9, 128, 4>(a, b, fstride, n);
    run_tile<7, 64, 2>(a, b, fstride, n);
    run_tile<1, 64, 2>(a, b, fstride, n);
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
