// Host <-> device copy paths for the one-shot C entry points (rcp_profile's matrix D2H, the
// readset's H2D): pageable vs hipHostRegister'ed caller memory vs pinned staging buffers with
// host threads copying out of them.  tools/pcie_bench [MB] [threads]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                             \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                 \
        }                                                                 \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(char* dst, const char* src, size_t n, int nt) {
    std::vector<std::thread> th;
    const size_t per = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const size_t a = t * per, b = std::min(n, a + per);
        if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
    }
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? atoll(argv[1]) : 1600;
    const int nt = argc > 2 ? atoi(argv[2]) : 8;
    const size_t n = mb << 20;
    char* d;
    CK(hipMalloc(&d, n));
    CK(hipMemset(d, 3, n));
    hipStream_t s[2];
    CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
    char* h = (char*)std::malloc(n);
    std::memset(h, 1, n);  // first touch outside the timing (R's allocMatrix memory is touched)
    const double gb = n / 1e9;
    double t;
    for (int rep = 0; rep < 2; ++rep) {
        t = now();
        CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
        std::printf("D2H pageable           %7.1f ms %6.1f GB/s\n", (now() - t) * 1e3, gb / (now() - t));
    }
    t = now();
    CK(hipHostRegister(h, n, hipHostRegisterDefault));
    const double treg = now() - t;
    t = now();
    CK(hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    const double tcp = now() - t;
    t = now();
    CK(hipHostUnregister(h));
    const double tun = now() - t;
    std::printf("D2H registered         %7.1f ms %6.1f GB/s (+ register %.1f ms, unregister %.1f ms)\n", tcp * 1e3,
                gb / tcp, treg * 1e3, tun * 1e3);
    char* pin;
    CK(hipHostMalloc(&pin, n, 0));
    for (int rep = 0; rep < 2; ++rep) {
        t = now();
        CK(hipMemcpy(pin, d, n, hipMemcpyDeviceToHost));
        std::printf("D2H pinned             %7.1f ms %6.1f GB/s\n", (now() - t) * 1e3, gb / (now() - t));
    }
    for (int rep = 0; rep < 2; ++rep) {
        t = now();
        CK(hipMemcpy(d, pin, n, hipMemcpyHostToDevice));
        std::printf("H2D pinned             %7.1f ms %6.1f GB/s\n", (now() - t) * 1e3, gb / (now() - t));
    }
    for (int rep = 0; rep < 2; ++rep) {
        t = now();
        CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
        std::printf("H2D pageable           %7.1f ms %6.1f GB/s\n", (now() - t) * 1e3, gb / (now() - t));
    }
    // staged: chunk k D2H into pinned buffer k%2 on stream k%2 while host threads copy chunk k-1 out
    for (size_t chunk_mb : {16, 64}) {
        for (int threads : {4, nt}) {
            const size_t ch = chunk_mb << 20;
            const size_t nch = (n + ch - 1) / ch;
            hipEvent_t ev[2];
            CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
            t = now();
            for (size_t k = 0; k <= nch; ++k) {
                if (k < nch) {
                    const size_t a = k * ch, b = std::min(n, a + ch);
                    CK(hipMemcpyAsync(pin + (k % 2) * ch, d + a, b - a, hipMemcpyDeviceToHost, s[k % 2]));
                    CK(hipEventRecord(ev[k % 2], s[k % 2]));
                }
                if (k > 0) {
                    const size_t j = k - 1, a = j * ch, b = std::min(n, a + ch);
                    CK(hipEventSynchronize(ev[j % 2]));
                    par_copy(h + a, pin + (j % 2) * ch, b - a, threads);
                }
            }
            std::printf("D2H staged %3zu MB x2, %2d thr %7.1f ms %6.1f GB/s\n", chunk_mb, threads, (now() - t) * 1e3,
                        gb / (now() - t));
            // H2D staged: host threads fill buffer k%2, then async copy
            t = now();
            for (size_t k = 0; k < nch; ++k) {
                const size_t a = k * ch, b = std::min(n, a + ch);
                if (k >= 2) CK(hipEventSynchronize(ev[k % 2]));
                par_copy(pin + (k % 2) * ch, h + a, b - a, threads);
                CK(hipMemcpyAsync(d + a, pin + (k % 2) * ch, b - a, hipMemcpyHostToDevice, s[k % 2]));
                CK(hipEventRecord(ev[k % 2], s[k % 2]));
            }
            CK(hipStreamSynchronize(s[0]));
            CK(hipStreamSynchronize(s[1]));
            std::printf("H2D staged %3zu MB x2, %2d thr %7.1f ms %6.1f GB/s\n", chunk_mb, threads, (now() - t) * 1e3,
                        gb / (now() - t));
        }
    }
    std::printf("host threads: hardware_concurrency %u\n", std::thread::hardware_concurrency());
    return 0;
}
