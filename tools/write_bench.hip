// Micro-benchmark: write an R x B fp64 column-major matrix with T-row column segments.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int T>
__global__ void wr(double* out, int R, int B) {
    const int tile = blockIdx.x;
    const int ii = threadIdx.x % T;
    const int kstep = 256 / T;
    const int r = tile * T + ii;
    if (r >= R) return;
    for (int k = threadIdx.x / T; k < B; k += kstep) out[(size_t)k * R + r] = (double)(k + r);
}

// same with non-temporal stores (what the pileup epilogue issues)
template <int T>
__global__ void wr_nt(double* out, int R, int B) {
    const int tile = blockIdx.x;
    const int ii = threadIdx.x % T;
    const int kstep = 256 / T;
    const int r = tile * T + ii;
    if (r >= R) return;
    for (int k = threadIdx.x / T; k < B; k += kstep) __builtin_nontemporal_store((double)(k + r), out + (size_t)k * R + r);
}

// T-row segments, but the two workgroups writing the two halves of each 2T-row segment
// are blocks b and b + 8 (same XCD under round-robin dispatch)
template <int T>
__global__ void wr_pair(double* out, int R, int B) {
    const int G = blockIdx.x / 16, x = blockIdx.x % 16;
    const int m = x / 8, s = x % 8;
    const int pair = G * 8 + s;
    const int ii = threadIdx.x % T;
    const int kstep = 256 / T;
    const int r = pair * 2 * T + m * T + ii;
    if (r >= R) return;
    for (int k = threadIdx.x / T; k < B; k += kstep) out[(size_t)k * R + r] = (double)(k + r);
}

// mixed stream: each 16-row tile reads its own contiguous slice of `in` (the reads the
// pileup kernel streams) and then writes its 16-row column segments
__global__ void rw16(const int2* __restrict__ in, size_t per_tile, double* out, int R, int B) {
    const int tile = blockIdx.x;
    const int ii = threadIdx.x % 16;
    const int r = tile * 16 + ii;
    const int2* src = in + (size_t)tile * per_tile;
    int acc = 0;
    for (size_t q = threadIdx.x; q < per_tile; q += 256) {
        const int2 v = src[q];
        acc += v.x ^ v.y;
    }
    if (r >= R) return;
    for (int k = threadIdx.x / 16; k < B; k += 16)
        __builtin_nontemporal_store((double)(k + r + (acc & 1)), out + (size_t)k * R + r);
}

// row-major reference (fully coalesced)
__global__ void wr_rm(double* out, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = (double)i;
}

template <int T>
float run(double* d, int R, int B) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(wr<T>, dim3((R + T - 1) / T), dim3(256), 0, 0, d, R, B);
    hipEventRecord(a);
    for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr<T>, dim3((R + T - 1) / T), dim3(256), 0, 0, d, R, B);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    const int R = 200000, B = 1000;
    double* d;
    hipMalloc(&d, (size_t)R * B * 8);
    const double gb = (double)R * B * 8 / 1e9;
    float t;
    t = run<4>(d, R, B);  printf("T=4   %.3f ms %.0f GB/s\n", t, gb / t * 1e3);
    {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        const int pairs = (R + 15) / 16, grid = ((pairs + 7) / 8) * 16;
        hipLaunchKernelGGL(wr_pair<8>, dim3(grid), dim3(256), 0, 0, d, R, B);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_pair<8>, dim3(grid), dim3(256), 0, 0, d, R, B);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("T=8 paired b/b+8  %.3f ms %.0f GB/s\n", ms / 10, gb / (ms / 10) * 1e3);
    }
    t = run<8>(d, R, B);  printf("T=8   %.3f ms %.0f GB/s\n", t, gb / t * 1e3);
    t = run<16>(d, R, B); printf("T=16  %.3f ms %.0f GB/s\n", t, gb / t * 1e3);
    t = run<32>(d, R, B); printf("T=32  %.3f ms %.0f GB/s\n", t, gb / t * 1e3);
    t = run<64>(d, R, B); printf("T=64  %.3f ms %.0f GB/s\n", t, gb / t * 1e3);
    {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(wr_nt<16>, dim3((R + 15) / 16), dim3(256), 0, 0, d, R, B);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_nt<16>, dim3((R + 15) / 16), dim3(256), 0, 0, d, R, B);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("T=16 nt  %.3f ms %.0f GB/s\n", ms / 10, gb / (ms / 10) * 1e3);
    }
    {
        const size_t tiles = (R + 15) / 16, per_tile = 663000000 / 8 / tiles;
        int2* in;
        hipMalloc(&in, tiles * per_tile * 8);
        hipMemset(in, 1, tiles * per_tile * 8);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(rw16, dim3(tiles), dim3(256), 0, 0, in, per_tile, d, R, B);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(rw16, dim3(tiles), dim3(256), 0, 0, in, per_tile, d, R, B);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("read 663 MB + write T=16 nt  %.3f ms %.0f GB/s\n", ms / 10, (gb + 0.663) / (ms / 10) * 1e3);
        hipFree(in);
    }
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(wr_rm, dim3(4096), dim3(256), 0, 0, d, (size_t)R * B);
    hipEventRecord(a);
    for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_rm, dim3(4096), dim3(256), 0, 0, d, (size_t)R * B);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("row-major stream %.3f ms %.0f GB/s\n", ms / 10, gb / (ms / 10) * 1e3);
    return 0;
}
