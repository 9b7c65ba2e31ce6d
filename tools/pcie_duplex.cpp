// Both PCIe directions at once, and the host memory traffic behind a staged copy:
//   1. pinned H2D alone, pinned D2H alone, both at once (two streams; no host memcpy)
//   2. host memcpy bandwidth (pageable -> pageable), T threads, plain and non-temporal stores
//   3. staged H2D + staged D2H at once (pinned double buffers + host memcpy threads, as
//      recoup_amd/csrc/rcp_stage.cpp does)
// tools/pcie_duplex [MB] [threads]
#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                   \
    do {                                                        \
        hipError_t e_ = (x);                                    \
        if (e_ != hipSuccess) {                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                       \
        }                                                       \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void copy_nt(char* dst, const char* src, size_t n) {
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
        const __m128i d = _mm_loadu_si128((const __m128i*)(src + i + 48));
        _mm_stream_si128((__m128i*)(dst + i), a);
        _mm_stream_si128((__m128i*)(dst + i + 16), b);
        _mm_stream_si128((__m128i*)(dst + i + 32), c);
        _mm_stream_si128((__m128i*)(dst + i + 48), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

static void par(int nt, size_t n, bool nt_store, char* dst, const char* src) {
    std::vector<std::thread> th;
    const size_t per = ((n + nt - 1) / nt + 4095) & ~size_t(4095);
    for (int t = 0; t < nt; ++t) {
        const size_t a = std::min(n, t * per), b = std::min(n, a + per);
        if (a < b)
            th.emplace_back([=] {
                if (nt_store) copy_nt(dst + a, src + a, b - a);
                else std::memcpy(dst + a, src + a, b - a);
            });
    }
    for (auto& x : th) x.join();
}

// chunked pinned copies on one stream (64 MB, as the stager's DMA chunks)
static void dma(char* dev, char* pin, size_t n, bool h2d, hipStream_t s) {
    const size_t ch = size_t(64) << 20;
    for (size_t a = 0; a < n; a += ch) {
        const size_t len = std::min(ch, n - a);
        if (h2d) CK(hipMemcpyAsync(dev + a, pin + (a % (2 * ch)), len, hipMemcpyHostToDevice, s));
        else CK(hipMemcpyAsync(pin + (a % (2 * ch)), dev + a, len, hipMemcpyDeviceToHost, s));
    }
}

// staged copy as rcp_stage.cpp: double buffer, nt memcpy threads fill / drain
static void staged(char* dev, char* host, char* pin2, size_t n, bool h2d, int nt, hipStream_t s, hipEvent_t* ev) {
    const size_t ch = size_t(64) << 20;
    const size_t nch = (n + ch - 1) / ch;
    if (h2d) {
        for (size_t k = 0; k < nch; ++k) {
            const int b = (int)(k & 1);
            const size_t a0 = k * ch, len = std::min(ch, n - a0);
            if (k >= 2) CK(hipEventSynchronize(ev[b]));
            par(nt, len, true, pin2 + b * ch, host + a0);
            CK(hipMemcpyAsync(dev + a0, pin2 + b * ch, len, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[b], s));
        }
    } else {
        for (size_t k = 0; k <= nch; ++k) {
            if (k < nch) {
                const int b = (int)(k & 1);
                const size_t a0 = k * ch, len = std::min(ch, n - a0);
                CK(hipMemcpyAsync(pin2 + b * ch, dev + a0, len, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[b], s));
            }
            if (k > 0) {
                const size_t j = k - 1;
                const int b = (int)(j & 1);
                const size_t a0 = j * ch, len = std::min(ch, n - a0);
                CK(hipEventSynchronize(ev[b]));
                par(nt, len, true, host + a0, pin2 + b * ch);
            }
        }
    }
    CK(hipStreamSynchronize(s));
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? atoll(argv[1]) : 1024;
    const int nt = argc > 2 ? atoi(argv[2]) : 4;
    const size_t n = mb << 20;
    const double gb = n / 1e9;
    char *d_up, *d_down, *pin_up, *pin_down, *pin2_up, *pin2_down;
    CK(hipMalloc(&d_up, n));
    CK(hipMalloc(&d_down, n));
    CK(hipMemset(d_down, 3, n));
    const size_t ch2 = size_t(128) << 20;
    CK(hipHostMalloc((void**)&pin_up, ch2, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin_down, ch2, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin2_up, ch2, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin2_down, ch2, hipHostMallocDefault));
    char* h_src = (char*)std::malloc(n);
    char* h_dst = (char*)std::malloc(n);
    std::memset(h_src, 1, n);
    std::memset(h_dst, 2, n);
    hipStream_t s[2];
    CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
    hipEvent_t ev_up[2], ev_down[2];
    for (int b = 0; b < 2; ++b) {
        CK(hipEventCreateWithFlags(&ev_up[b], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_down[b], hipEventDisableTiming));
    }
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        dma(d_up, pin_up, n, true, s[0]);
        CK(hipStreamSynchronize(s[0]));
        const double th2d = now() - t;
        t = now();
        dma(d_down, pin_down, n, false, s[1]);
        CK(hipStreamSynchronize(s[1]));
        const double td2h = now() - t;
        t = now();
        dma(d_up, pin_up, n, true, s[0]);
        dma(d_down, pin_down, n, false, s[1]);
        CK(hipStreamSynchronize(s[0]));
        const double tu = now() - t;
        CK(hipStreamSynchronize(s[1]));
        const double tb = now() - t;
        std::printf("pinned: h2d %.1f GB/s, d2h %.1f GB/s, both: %.1f ms (h2d done %.1f ms) = %.1f GB/s total\n",
                    gb / th2d, gb / td2h, tb * 1e3, tu * 1e3, 2 * gb / tb);
    }
    for (int k : {1, 2, 4, 8, 16}) {
        for (int ntst = 0; ntst < 2; ++ntst) {
            par(k, n, ntst, h_dst, h_src);
            const double t = now();
            par(k, n, ntst, h_dst, h_src);
            const double dt = now() - t;
            std::printf("host memcpy %2d threads %s: %.1f GB/s copied (%.1f GB/s of traffic incl. RFO)\n", k,
                        ntst ? "nt   " : "plain", gb / dt, gb * (ntst ? 2 : 3) / dt);
        }
    }
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        staged(d_up, h_src, pin2_up, n, true, nt, s[0], ev_up);
        const double tu = now() - t;
        t = now();
        staged(d_down, h_dst, pin2_down, n, false, nt, s[1], ev_down);
        const double td = now() - t;
        t = now();
        std::thread a([&] { staged(d_up, h_src, pin2_up, n, true, nt, s[0], ev_up); });
        std::thread b([&] { staged(d_down, h_dst, pin2_down, n, false, nt, s[1], ev_down); });
        a.join();
        b.join();
        const double tb = now() - t;
        std::printf("staged (%d threads each): h2d %.1f GB/s, d2h %.1f GB/s, both %.1f ms = %.1f GB/s total\n", nt,
                    gb / tu, gb / td, tb * 1e3, 2 * gb / tb);
    }
    return 0;
}
