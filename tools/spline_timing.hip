// Cost of splitVector's spline rows in isolation (rcp_splitvector.h): one block per row with the
// spline arrays in LDS, as rcp_interp_kernel runs them, without the pileup.  Prints the kernel time
// for B rows of L positions into N bins, and the cycles thread 0 spends in the fmm chains.
//   tools/spline_timing [B] [L] [N]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../recoup_amd/csrc/rcp_splitvector.h"

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                 \
        }                                                                 \
    } while (0)

__global__ void __launch_bounds__(256) spline_rows(int L, int n, const double* tb, double* out, long long* cyc,
                                                   int phase) {
    extern __shared__ double sm[];
    double* x = sm;  // x (L + 1) | b, c, d (L + 1 each)
    for (int i = threadIdx.x; i < L; i += blockDim.x) x[i] = (double)((i * 7919 + blockIdx.x * 31) % 1000) * 0.25;
    __syncthreads();
    const long long t0 = clock64();
    if (phase == 0) {
        double* b = x + L + 1;
        fmm_spline_block(L, x, b, b + L + 1, b + 2 * (L + 1), tb);
    } else {
        interp_finish(1, L, n, x, nullptr, tb, out + blockIdx.x, gridDim.x);
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// cycles per step of a dependent FP64 chain in one lane (mul + sub, no contraction), for scale
#pragma clang fp contract(off)
__global__ void chain_latency(double a, double b, int steps, double* out, long long* cyc) {
    double x = (double)threadIdx.x;
    const long long t0 = clock64();
    for (int i = 0; i < steps; ++i) x = b - a * x;
    const long long t1 = clock64();
    if (threadIdx.x == 0) {
        out[0] = x;
        cyc[0] = t1 - t0;
    }
}
#pragma clang fp contract(on)

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1555;
    const int L = argc > 2 ? atoi(argv[2]) : 300;
    const int n = argc > 3 ? atoi(argv[3]) : 500;
    std::vector<double> tb(2 * (L + 1));
    double bp = -1.0;
    tb[1] = bp;
    for (size_t i = 1; 2 * i + 1 < tb.size(); ++i) {
        const double t = 1.0 / bp;
        bp = 4.0 - t;
        tb[2 * i] = t;
        tb[2 * i + 1] = bp;
    }
    double *d_tb, *d_out;
    long long* d_cyc;
    CK(hipMalloc(&d_tb, 8 * tb.size()));
    CK(hipMalloc(&d_out, 8 * (size_t)B * n));
    CK(hipMalloc(&d_cyc, 8 * (size_t)B));
    CK(hipMemcpy(d_tb, tb.data(), 8 * tb.size(), hipMemcpyHostToDevice));
    const size_t lds = 8 * (size_t)(4 * (L + 1) + n + 8);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int phase = 0; phase < 2; ++phase) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(spline_rows, dim3(B), dim3(256), lds, 0, L, n, d_tb, d_out, d_cyc, phase);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::vector<long long> cyc(B);
            CK(hipMemcpy(cyc.data(), d_cyc, 8 * (size_t)B, hipMemcpyDeviceToHost));
            long long mx = 0, sum = 0;
            for (long long c : cyc) {
                mx = std::max(mx, c);
                sum += c;
            }
            std::printf("%s B=%d L=%d n=%d: kernel %.1f us, cycles per block mean %lld max %lld\n",
                        phase ? "spline + eval" : "fmm chains  ", B, L, n, ms * 1e3, sum / B, mx);
        }
    }
    {
        const int steps = 10000;
        hipLaunchKernelGGL(chain_latency, dim3(1), dim3(64), 0, 0, 0.25, 1.5, steps, d_out, d_cyc);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(chain_latency, dim3(1), dim3(64), 0, 0, 0.25, 1.5, steps, d_out, d_cyc);
        long long c = 0;
        CK(hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost));
        std::printf("dependent fp64 mul + sub: %.1f cycles per step\n", (double)c / steps);
    }
    return 0;
}
