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

// 16 B per lane: lane writes rows 2 ii, 2 ii + 1 of a column (T rows per column segment)
template <int T>
__global__ void wr_v2(double* out, int R, int B) {
    const int tile = blockIdx.x;
    constexpr int H = T / 2;  // lanes per column segment
    const int ii = threadIdx.x % H;
    const int kstep = 256 / H;
    const int r = tile * T + 2 * ii;
    if (r + 1 >= R) return;
    for (int k = threadIdx.x / H; k < B; k += kstep)
        *reinterpret_cast<double2*>(out + (size_t)k * R + r) = make_double2((double)(k + r), (double)(k + r + 1));
}

// row-major stream, 16 B per lane, persistent grid
__global__ void wr_rm2(double* out, size_t n) {
    double2* o = reinterpret_cast<double2*>(out);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n / 2; i += (size_t)gridDim.x * 256)
        o[i] = make_double2((double)i, (double)(i + 1));
}

// row-major stream variants (what does the runtime's fill do that a plain stream does not?)
//  V 0: 16 B/lane, 4 coalesced stores per iteration (stride = grid); V 1: same with constant data;
//  V 2: 64 B contiguous per lane (4 x 16 B); V 3: non-temporal 16 B stores; V 4: 16 B/lane with
//  dwordx4 of int (no fp conversion)
template <int V>
__global__ void wr_rmv(double* out, size_t n) {
    uint4* o = reinterpret_cast<uint4*>(out);
    const size_t n16 = n / 2;
    const size_t G = (size_t)gridDim.x * blockDim.x;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (V == 2) {
        for (size_t i = t * 4; i + 3 < n16; i += G * 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) o[i + u] = make_uint4((uint32_t)i, u, 1u, 2u);
        }
        return;
    }
    for (size_t i = t; i < n16; i += 4 * G) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = i + u * G;
            if (j < n16) {
                const uint4 v = V == 1 ? make_uint4(7u, 7u, 7u, 7u) : make_uint4((uint32_t)j, (uint32_t)(j >> 7), 3u, (uint32_t)u);
                if (V == 3) {
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u w = {v.x, v.y, v.z, v.w};
                    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(o + j));
                }
                else o[j] = v;
            }
        }
    }
}

// one 16-B store per thread, a block per (64-row tile, 8 columns) or per 4 KB of row-major
// output: the grid is the whole output (what the runtime's fill kernel does)
template <int CM>
__global__ void wr_one(double* out, int R, int B) {
    if (CM) {
        const int nt = (R + 63) / 64;
        const int tile = blockIdx.x % nt, cg = blockIdx.x / nt;
        const int c = cg * 8 + (threadIdx.x >> 5);
        const int r = tile * 64 + 2 * (threadIdx.x & 31);
        if (c < B && r + 1 < R)
            *reinterpret_cast<double2*>(out + (size_t)c * R + r) = make_double2((double)r, (double)c);
    } else {
        const size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
        if (j < (size_t)R * B / 2) reinterpret_cast<double2*>(out)[j] = make_double2((double)j, 1.0);
    }
}

// column-major, TT-row column segments written by one block at once (16 B per thread)
template <int TT>
__global__ void wr_seg(double* out, int R, int B) {
    constexpr int LPC = TT / 2;                         // threads per column segment
    constexpr int CPB = 256 / LPC > 0 ? 256 / LPC : 1;  // columns per block pass
    const int nt = (R + TT - 1) / TT;
    const int tile = blockIdx.x % nt, cg = blockIdx.x / nt;
    for (int t = threadIdx.x; t < CPB * LPC; t += 256) {
        const int c = cg * CPB + t / LPC;
        const int r = tile * TT + 2 * (t % LPC);
        if (c < B && r + 1 < R)
            *reinterpret_cast<double2*>(out + (size_t)c * R + r) = make_double2((double)r, (double)c);
    }
}
template <int TT>
void run_seg(double* d, int R, int B, double gb) {
    constexpr int LPC = TT / 2;
    constexpr int CPB = 256 / LPC > 0 ? 256 / LPC : 1;
    const unsigned grid = (unsigned)(((R + TT - 1) / TT) * ((B + CPB - 1) / CPB));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(wr_seg<TT>, dim3(grid), dim3(256), 0, 0, d, R, B);
    hipEventRecord(a);
    for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_seg<TT>, dim3(grid), dim3(256), 0, 0, d, R, B);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("col-major segments of %d rows, one block at once  %.3f ms %.0f GB/s\n", TT, ms / 10, gb / (ms / 10) * 1e3);
}

template <int V>
void run_rmv(double* d, size_t n, int grid, int block, double gb) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(wr_rmv<V>, dim3(grid), dim3(block), 0, 0, d, n);
    hipEventRecord(a);
    for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_rmv<V>, dim3(grid), dim3(block), 0, 0, d, n);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("rm V%d grid %d x %d  %.3f ms %.0f GB/s\n", V, grid, block, ms / 10, gb / (ms / 10) * 1e3);
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
    for (int T2 : {16, 32, 64}) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        auto k = T2 == 16 ? wr_v2<16> : T2 == 32 ? wr_v2<32> : wr_v2<64>;
        hipLaunchKernelGGL(k, dim3((R + T2 - 1) / T2), dim3(256), 0, 0, d, R, B);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(k, dim3((R + T2 - 1) / T2), dim3(256), 0, 0, d, R, B);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("T=%d 16B/lane  %.3f ms %.0f GB/s\n", T2, ms / 10, gb / (ms / 10) * 1e3);
    }
    for (int g : {2048, 4096, 16384}) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(wr_rm2, dim3(g), dim3(256), 0, 0, d, (size_t)R * B);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(wr_rm2, dim3(g), dim3(256), 0, 0, d, (size_t)R * B);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("row-major stream 16B/lane grid %d  %.3f ms %.0f GB/s\n", g, ms / 10, gb / (ms / 10) * 1e3);
    }
    {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(d), 7, (size_t)R * B * 2);
        hipEventRecord(a);
        for (int it = 0; it < 10; ++it) hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(d), 7, (size_t)R * B * 2);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("hipMemsetD32  %.3f ms %.0f GB/s\n", ms / 10, gb / (ms / 10) * 1e3);
    }
    {
        const size_t n = (size_t)R * B;
        for (int g : {2048, 8192, 32768}) {
            run_rmv<0>(d, n, g, 256, gb);
            run_rmv<1>(d, n, g, 256, gb);
            run_rmv<2>(d, n, g, 256, gb);
            run_rmv<3>(d, n, g, 256, gb);
        }
        for (int cm = 0; cm < 2; ++cm) {
            const unsigned grid = cm ? (unsigned)(((R + 63) / 64) * ((B + 7) / 8)) : (unsigned)((n / 2 + 255) / 256);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            auto k = cm ? wr_one<1> : wr_one<0>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, R, B);
            hipEventRecord(a);
            for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, R, B);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            printf("one store per thread %s grid %u  %.3f ms %.0f GB/s\n", cm ? "col-major T=64" : "row-major", grid, ms / 10, gb / (ms / 10) * 1e3);
        }
        run_seg<64>(d, R, B, gb);
        run_seg<128>(d, R, B, gb);
        run_seg<256>(d, R, B, gb);
        run_seg<512>(d, R, B, gb);
        run_rmv<0>(d, n, 4096, 1024, gb);
        run_rmv<1>(d, n, 4096, 1024, gb);
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
