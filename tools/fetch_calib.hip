// PMC calibration for the pileup kernel's access shapes (MI355X_MICROARCH.md documents the
// FETCH_SIZE correction only for 16-B-per-lane reads; the pileup streams 8-B int2 reads (4-B
// starts for uniform-width readsets) and
// writes 8-B fp64 non-temporal stores in 128-B column segments).
//
//   fetch_calib          runs each kernel 3 times over a 2 GiB buffer (far beyond L2 + MALL)
// Profile with separate passes, e.g.
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o p -- tools/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o p -- tools/fetch_calib
// and divide the known bytes (printed) by the counter (KiB) per dispatch: tools/pmc_calib.py.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void read8(const int2* __restrict__ in, size_t n, int* __restrict__ sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const long long v = __builtin_nontemporal_load(reinterpret_cast<const long long*>(in) + i);
        acc += (int)v ^ (int)(v >> 32);
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void read16(const int4* __restrict__ in, size_t n, int* __restrict__ sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 v = in[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

// plain int2 loads (what the pileup issues: global_load_dwordx2)
__global__ void read8_plain(const int2* __restrict__ in, size_t n, int* __restrict__ sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int2 v = in[i];
        acc += v.x ^ v.y;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

// plain int32 loads (the lean pileup over a uniform-width readset's starts: global_load_dword)
__global__ void read4_plain(const int* __restrict__ in, size_t n, int* __restrict__ sink) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += in[i];
    if (acc == 0x7fffffff) sink[0] = acc;
}

// column-major fp64 matrix, 16-row column segments, non-temporal 8-B stores (the epilogue)
__global__ void write8_seg16(double* out, int R, int B) {
    const int r = blockIdx.x * 16 + threadIdx.x % 16;
    if (r >= R) return;
    for (int k = threadIdx.x / 16; k < B; k += 16) __builtin_nontemporal_store((double)(k + r), out + (size_t)k * R + r);
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    void* buf;
    int* sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
    const int R = 262144, B = bytes / 8 / R;
    for (int it = 0; it < 3; ++it) {
        hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, (const int2*)buf, bytes / 8, sink);
        hipLaunchKernelGGL(read8_plain, dim3(4096), dim3(256), 0, 0, (const int2*)buf, bytes / 8, sink);
        hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, (const int4*)buf, bytes / 16, sink);
        hipLaunchKernelGGL(read4_plain, dim3(4096), dim3(256), 0, 0, (const int*)buf, bytes / 4, sink);
        hipLaunchKernelGGL(write8_seg16, dim3(R / 16), dim3(256), 0, 0, (double*)buf, R, B);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"bytes_per_dispatch\": %zu}\n", bytes);
    return 0;
}
