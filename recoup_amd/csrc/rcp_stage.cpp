// rcp_stage.cpp -- pinned double-buffered staging of pageable host memory (rcp_stage.h).
//
// Per device and direction: two 64 MB pinned buffers, one HIP event each, and a small pool of
// host threads that memcpy between the caller's memory and the pinned buffer.  D2H: chunk k is
// DMA'd into buffer k % 2 while the threads drain chunk k - 1; H2D: the threads fill chunk k
// while the DMA engine uploads chunk k - 1.  A mutex per (device, direction) serialises users of
// one set of buffers; the two directions of a device proceed in parallel (PCIe is full duplex:
// one sample's upload beside another's download, rcp_profile_samples_reads), and so do devices
// (rcp_profile_multi drives one host thread per GPU).
#include "rcp_stage.h"

#include "rcp_pack.h"

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

extern "C" {
int rcp_pack_block(void);
hipError_t rcp_launch_unpack_i32(const void* src, int64_t n, int32_t* dst, hipStream_t stream);
hipError_t rcp_launch_unpack_strand(const void* src, int64_t n, int8_t* dst, hipStream_t stream);
hipError_t rcp_launch_unpack_code8(const void* src, int64_t n, int32_t* dst, hipStream_t stream);
hipError_t rcp_launch_pack_i32(const int32_t* src, int64_t n, void* dst, hipStream_t stream);
}

namespace rcp {
namespace {

constexpr size_t kChunk = size_t(64) << 20;  // 64 MB: 51-54 GB/s vs 41 GB/s at 16 MB (pcie.log)
constexpr size_t kDirect = size_t(4) << 20;  // below this, a plain hipMemcpy
// memcpy threads per direction: 4 saturate one direction of an x16 link alone (pcie.log), but
// with both directions busy the host memory traffic (3 bytes per byte moved) needs 8 each to keep
// 86 GB/s in flight vs 55 with 4 (profiles/r05/pcie_duplex.log).  The download -- a profile's
// matrix, 1.6x a C4 sample's reads -- is the longer direction of a streamed sample: it gets more.
constexpr int kThreadsDir[2] = {8, 8};
constexpr int kMaxDevices = 64;

// A fixed pool: run(parts, fn) executes fn(0 .. parts - 1) on the workers and the caller.
class Pool {
  public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void run(int parts, const std::function<void(int)>& fn) {
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            parts_ = parts;
            next_ = 0;
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return done_ == parts_; });
        fn_ = nullptr;
    }

  private:
    void work() {
        for (;;) {
            int i;
            const std::function<void(int)>* fn;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!fn_ || next_ >= parts_) return;
                i = next_++;
                fn = fn_;
            }
            (*fn)(i);
            std::lock_guard<std::mutex> g(mu_);
            if (++done_ == parts_) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* fn_ = nullptr;
    int parts_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct Stager {
    std::mutex mu;
    bool init = false, ok = false;
    char* pin[2] = {nullptr, nullptr};
    // blocking-sync events: a thread waiting for a DMA sleeps instead of spinning -- the box gives
    // a process 16 cores of CPU time (cgroup quota), and spinning waiters next to the memcpy
    // threads ran it out (10-ms stalls of every thread until the next quota period)
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipEvent_t done = nullptr;
    std::unique_ptr<Pool> pool;
    char* dev[2] = {nullptr, nullptr};  // device buffers of packed chunks: H2D landing (decoded into place),
                                        // D2H packing (rcp_pack_i32_kernel)
};

// The host -> device lane of this thread (H2dLane): lane 1 has its own pinned buffers, landing
// buffers and copy threads, so two uploads of one device run at once
thread_local int t_h2d_lane = 0;

// Process lifetime: the pinned buffers are returned to the OS at exit (freeing them from a
// static destructor could run after the HIP runtime is gone).
Stager* stager(int device, int dir) {  // dir 0: host -> device (this thread's lane), 1: device -> host
    static Stager* s = new Stager[3 * kMaxDevices];
    const int k = dir == 0 && t_h2d_lane ? 2 : dir;
    return device >= 0 && device < kMaxDevices ? &s[3 * device + k] : nullptr;
}

bool ready(Stager* s, int dir) {  // under s->mu, on the device
    if (s->init) return s->ok;
    s->init = true;
    for (int b = 0; b < 2; ++b) {
        if (hipHostMalloc(reinterpret_cast<void**>(&s->pin[b]), kChunk, hipHostMallocDefault) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&s->ev[b], hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
            return false;
    }
    if (hipEventCreateWithFlags(&s->done, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) return false;
    try {
        int nt = kThreadsDir[dir];
        // (RCP_H2D_THREADS / RCP_D2H_THREADS: diagnostics A/B of the copy threads per direction)
        if (const char* e = std::getenv(dir == 0 ? "RCP_H2D_THREADS" : "RCP_D2H_THREADS"))
            nt = std::min(32, std::max(1, std::atoi(e)));
        s->pool.reset(new Pool(nt - 1));
    } catch (const std::exception&) {
        return false;
    }
    s->ok = true;
    return true;
}

// RCP_TRACE=1 in the environment: one stderr line per staged copy (direction, bytes, time waiting
// for the direction's buffers, copy time) -- diagnostics of the PCIe pipelines, off by default
bool trace() { return std::getenv("RCP_TRACE") != nullptr; }  // (read per call: tests set it around one call)
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The direction's buffers: a copy below kShared does not wait for them when another thread holds
// them (the lock comes back unowned) but goes through HIP's own staging -- a plan's table upload
// need not queue behind the next sample's multi-GB read upload
constexpr size_t kShared = size_t(16) << 20;
std::unique_lock<std::mutex> take(Stager* st, size_t bytes) {
    if (bytes < kShared) {
        std::unique_lock<std::mutex> g(st->mu, std::try_to_lock);
        return g;
    }
    return std::unique_lock<std::mutex>(st->mu);
}

// memcpy with non-temporal 16-B stores: the destination lines are not read first (no
// read-for-ownership) and do not evict the other direction's working set -- the host memory
// traffic of a staged copy is the DMA's plus one read and one write per byte
void copy_nt(char* dst, const char* src, size_t n) {
    if (n < 256) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    for (; i + 16 <= n; i += 16)
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i)));
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

// Chunk size of one staged copy: up to the 64 MB buffers, but a copy of less than 256 MB in four
// chunks at least (4 MB minimum), so that the host memcpy of one chunk runs beside the DMA of
// another -- a 50 MB copy in one chunk does them one after the other (24 GB/s)
size_t chunk_of(size_t bytes) {
    const size_t quarter = ((bytes / 4) + (size_t(1) << 20) - 1) & ~((size_t(1) << 20) - 1);
    return std::min(kChunk, std::max(size_t(4) << 20, quarter));
}

// A chunk is cut into kParts 4 KB-aligned parts taken by the threads as they come free: a
// thread descheduled for a while (the box's cores are shared with the pipeline's own threads)
// holds up 2 MB, not a whole thread's share of the chunk.
constexpr int kParts = 32;
inline void part_range(size_t n, int i, size_t* a, size_t* b) {
    const size_t per = ((n + kParts - 1) / kParts + 4095) & ~size_t(4095);
    *a = std::min(n, per * (size_t)i);
    *b = std::min(n, *a + per);
}

// dst[i] = q[i] * scale / div of row i (rows r .. r + n - 1 of a column; rcp_pack_kernel): the
// device's operations -- ((double)q * scale) * (1 / div) for a power of two, the correctly
// rounded quotient otherwise, +0.0 for a NULL row (div 0) -- with non-temporal stores
void expand_nt(double* dst, const uint32_t* q, const double* rd, const double* dv, bool all_pow2, double sc,
               size_t n) {
    auto one = [&](size_t i) -> double {
        const double x = (double)q[i] * sc;
        return dv[i] != 0.0 ? x / dv[i] : x * rd[i];
    };
    size_t i = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) && n) {
        dst[0] = one(0);
        i = 1;
    }
    if (all_pow2) {
        for (; i + 2 <= n; i += 2) {
            const __m128d x = _mm_set_pd((double)q[i + 1] * sc, (double)q[i] * sc);
            _mm_stream_pd(dst + i, _mm_mul_pd(x, _mm_loadu_pd(rd + i)));
        }
    } else {
        for (; i + 2 <= n; i += 2) _mm_stream_pd(dst + i, _mm_set_pd(one(i + 1), one(i)));
    }
    for (; i < n; ++i) dst[i] = one(i);
    _mm_sfence();
}

// device buffers of packed transfers, made on first use on the stager's device
bool ready_dev(Stager* s, int device) {
    if (s->dev[0] && s->dev[1]) return true;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || (cur != device && hipSetDevice(device) != hipSuccess)) {
        (void)hipGetLastError();
        return false;
    }
    bool ok = true;
    for (int b = 0; b < 2 && ok; ++b)
        if (!s->dev[b] && hipMalloc(reinterpret_cast<void**>(&s->dev[b]), kChunk) != hipSuccess) {
            (void)hipGetLastError();
            ok = false;
        }
    if (cur != device) (void)hipSetDevice(cur);
    return ok;
}

}  // namespace

bool trace_on() { return trace(); }
double trace_ms() { return now_ms(); }

H2dLane::H2dLane(int lane) : prev_(t_h2d_lane) { t_h2d_lane = lane; }
H2dLane::~H2dLane() { t_h2d_lane = prev_; }

hipError_t stage_h2d(void* dst, const void* src, size_t bytes, int device, hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    Stager* st = stager(device, 0);
    const double t0 = trace() ? now_ms() : 0.0;
    std::unique_lock<std::mutex> g;
    if (bytes >= kDirect && st) g = take(st, bytes);
    const double t1 = trace() ? now_ms() : 0.0;
    if (!g.owns_lock() || !ready(st, 0)) {
        hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream);
        e = e == hipSuccess ? hipStreamSynchronize(stream) : e;
        if (trace() && bytes >= kDirect)
            fprintf(stderr, "[stage] h2d %zu B direct %.2f ms\n", bytes, now_ms() - t1);
        return e;
    }
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    const size_t ch = chunk_of(bytes);
    const size_t nch = (bytes + ch - 1) / ch;
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < nch && e == hipSuccess; ++k) {
        const int b = (int)(k & 1);
        const size_t a0 = k * ch, len = std::min(ch, bytes - a0);
        if (k >= 2) e = hipEventSynchronize(st->ev[b]);  // the DMA out of this buffer is done
        if (e != hipSuccess) break;
        char* pin = st->pin[b];
        st->pool->run(kParts, [&](int i) {
            size_t a, z;
            part_range(len, i, &a, &z);
            if (z > a) copy_nt(pin + a, s + a0 + a, z - a);
        });
        e = hipMemcpyAsync(d + a0, pin, len, hipMemcpyHostToDevice, stream);
        if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
    }
    hipError_t e2 = hipEventRecord(st->done, stream);  // buffers free for the next user
    if (e2 == hipSuccess) e2 = hipEventSynchronize(st->done);
    if (trace()) fprintf(stderr, "[stage] h2d %zu B wait %.2f ms copy %.2f ms\n", bytes, t1 - t0, now_ms() - t1);
    return e != hipSuccess ? e : e2;
}

// ---- packed uploads: PCIe and host memory carry what the values need, the device restores them
// (rcp_kernels.hip rcp_unpack_*).  A chunk of m int32 values goes as [base x nb][slot x nb]
// [16-bit offsets x m (even)][raw blocks]: a block of B values spanning < 2^16 (coordinate-sorted
// starts: nearly every block) is its minimum + offsets, another one raw; a chunk with more raw
// blocks than its buffer holds goes plain.  Strand codes go four to a byte.
namespace {
constexpr size_t kPackMin = size_t(1) << 20;  // values; below this the plain copy

hipError_t h2d_packed(Stager* st, size_t n, size_t per_chunk, hipStream_t stream, const char* what,
                      const std::function<size_t(char* pin, size_t a0, size_t m, bool* plain)>& encode,
                      const std::function<hipError_t(const char* dev, char* dst_plain_chunk, size_t a0, size_t m,
                                                     size_t bytes, bool plain, hipStream_t s)>& land) {
    const double t1 = trace() ? now_ms() : 0.0;
    size_t raw_chunks = 0, sent = 0;
    const size_t nch = (n + per_chunk - 1) / per_chunk;
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < nch && e == hipSuccess; ++k) {
        const int b = (int)(k & 1);
        const size_t a0 = k * per_chunk, m = std::min(per_chunk, n - a0);
        if (k >= 2) e = hipEventSynchronize(st->ev[b]);  // buffer b's DMA (and the decode after it) queued before
        if (e != hipSuccess) break;
        bool plain = false;
        const size_t bytes = encode(st->pin[b], a0, m, &plain);
        raw_chunks += plain ? 1 : 0;
        sent += bytes;
        e = land(st->dev[b], st->pin[b], a0, m, bytes, plain, stream);
        if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
    }
    hipError_t e2 = hipEventRecord(st->done, stream);
    if (e2 == hipSuccess) e2 = hipEventSynchronize(st->done);
    if (trace())
        fprintf(stderr, "[stage] h2d-packed %s %zu values as %zu B (%zu of %zu chunks plain) %.2f ms\n", what, n, sent,
                raw_chunks, nch, now_ms() - t1);
    return e != hipSuccess ? e : e2;
}
}  // namespace

namespace {

// The packed upload of n int32 values a .. a + len - 1 of which `fill(tmp, a, len, &ok)` returns
// (the caller's array itself, or values it forms into tmp on the way: read widths; ok false: a
// value it cannot form).  A chunk whose
// first blocks are mostly raw (unsorted coordinates: no block spans < 2^16) goes plain at once
// rather than after half its blocks were copied into the raw area.  *unfit (may be NULL) is set
// when fill reports a value it cannot form (returns false): nothing usable was sent then.
hipError_t h2d_i32_from(int32_t* dst, size_t n, int device, hipStream_t stream, const char* what,
                        const std::function<const int32_t*(int32_t* tmp, size_t a, size_t len, bool* ok)>& fill,
                        bool* unfit) {
    Stager* st = stager(device, 0);
    std::unique_lock<std::mutex> g(st->mu);
    const size_t B = (size_t)rcp_pack_block();
    const size_t per_chunk = kChunk / 4;  // values: a plain chunk fills the buffer
    std::atomic<bool> bad_value{false};
    auto encode = [&](char* pin, size_t a0, size_t m, bool* plain) -> size_t {
        const size_t nb = (m + B - 1) / B;
        int32_t* base = reinterpret_cast<int32_t*>(pin);
        int32_t* slot = base + nb;
        uint16_t* off = reinterpret_cast<uint16_t*>(pin + 8 * nb);
        char* raw = pin + 8 * nb + 2 * ((m + 1) & ~size_t(1));
        const size_t cap = (kChunk - (size_t)(raw - pin)) / (4 * B);
        std::atomic<size_t> n_raw{0};
        std::atomic<bool> over{false};
        // probe: the chunk's first 16 blocks
        {
            alignas(16) int32_t v[1024];
            alignas(16) uint16_t tmp[1024 + 8];
            size_t probe_raw = 0;
            const size_t np = std::min<size_t>(16, nb);
            for (size_t b2 = 0; b2 < np; ++b2) {
                const size_t j0 = b2 * B, len = std::min(B, m - j0);
                int32_t lo = 0;
                bool ok = true;
                const int32_t* pv = fill(v, a0 + j0, len, &ok);
                if (!ok) bad_value.store(true);
                if (!rcp_pack_block16(pv, (int)len, tmp, &lo)) ++probe_raw;
            }
            if (np >= 8 && probe_raw * 4 >= np * 3) over.store(true);
        }
        if (!over.load())
            st->pool->run(kParts, [&](int i) {
                alignas(16) int32_t v[1024];
                alignas(16) uint16_t tmp[1024 + 8];
                const size_t b0 = nb * (size_t)i / kParts, b1 = nb * (size_t)(i + 1) / kParts;
                for (size_t b = b0; b < b1 && !over.load(std::memory_order_relaxed); ++b) {
                    const size_t j0 = b * B, len = std::min(B, m - j0);
                    bool ok = true;
                    const int32_t* pv = fill(v, a0 + j0, len, &ok);
                    if (!ok) bad_value.store(true, std::memory_order_relaxed);
                    int32_t lo = 0;
                    if (rcp_pack_block16(pv, (int)len, tmp, &lo)) {
                        base[b] = lo;
                        slot[b] = -1;
                        copy_nt(reinterpret_cast<char*>(off + j0), reinterpret_cast<const char*>(tmp), 2 * len);
                    } else {
                        const size_t q = n_raw.fetch_add(1, std::memory_order_relaxed);
                        if (q >= cap) {
                            over.store(true, std::memory_order_relaxed);
                            break;
                        }
                        base[b] = 0;
                        slot[b] = (int32_t)q;
                        copy_nt(raw + 4 * B * q, reinterpret_cast<const char*>(pv), 4 * len);
                    }
                }
            });
        if (over.load()) {  // too many raw blocks: the chunk as it is
            *plain = true;
            st->pool->run(kParts, [&](int i) {
                size_t a, z;
                part_range(m, i, &a, &z);
                if (z <= a) return;
                int32_t* out = reinterpret_cast<int32_t*>(pin) + a;
                bool ok = true;
                const int32_t* pv = fill(out, a0 + a, z - a, &ok);
                if (!ok) bad_value.store(true, std::memory_order_relaxed);
                if (pv != out) copy_nt(reinterpret_cast<char*>(out), reinterpret_cast<const char*>(pv), 4 * (z - a));
            });
            return 4 * m;
        }
        return (size_t)(raw - pin) + 4 * B * std::min(n_raw.load(), cap);
    };
    auto land = [&](const char* dev, char* pin, size_t a0, size_t m, size_t bytes, bool plain, hipStream_t s) {
        if (plain) return hipMemcpyAsync(dst + a0, pin, 4 * m, hipMemcpyHostToDevice, s);
        hipError_t e = hipMemcpyAsync(const_cast<char*>(dev), pin, bytes, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = rcp_launch_unpack_i32(dev, (int64_t)m, dst + a0, s);
        return e;
    };
    const hipError_t e = h2d_packed(st, n, per_chunk, stream, what, encode, land);
    if (unfit) *unfit = bad_value.load();
    return e;
}

bool packed_ready(Stager* st, int device) {  // (under st->mu)
    return ready(st, 0) && ready_dev(st, device);
}

}  // namespace

hipError_t stage_h2d_i32(int32_t* dst, const int32_t* src, size_t n, int device, hipStream_t stream) {
    Stager* st = stager(device, 0);
    if (n < kPackMin || !st) return stage_h2d(dst, src, 4 * n, device, stream);
    {
        std::unique_lock<std::mutex> g(st->mu);
        if (!packed_ready(st, device)) {
            g.unlock();
            return stage_h2d(dst, src, 4 * n, device, stream);
        }
    }
    return h2d_i32_from(dst, n, device, stream, "i32",
                        [&](int32_t*, size_t a, size_t, bool*) -> const int32_t* { return src + a; }, nullptr);
}

hipError_t stage_h2d_width(int32_t* dst, const int32_t* start, const int32_t* end, size_t n, int device,
                           hipStream_t stream, bool* unfit) {
    *unfit = false;
    Stager* st = stager(device, 0);
    bool packed = n >= kPackMin && st;
    if (packed) {
        std::unique_lock<std::mutex> g(st->mu);
        packed = packed_ready(st, device);
    }
    if (!packed) {
        // (few reads, or no landing buffers): the widths formed here, sent as they are
        std::vector<int32_t> w(n);
        for (size_t i = 0; i < n; ++i) {
            const int64_t x = (int64_t)end[i] - (int64_t)start[i] + 1;
            if (x < INT32_MIN || x > INT32_MAX) {
                *unfit = true;
                return hipSuccess;
            }
            w[i] = (int32_t)x;
        }
        return stage_h2d(dst, w.data(), 4 * n, device, stream);
    }
    return h2d_i32_from(dst, n, device, stream, "width",
                        [&](int32_t* out, size_t a, size_t len, bool* ok) -> const int32_t* {
                            bool good = true;
                            for (size_t j = 0; j < len; ++j) {
                                const int64_t x = (int64_t)end[a + j] - (int64_t)start[a + j] + 1;
                                good = good && x >= INT32_MIN && x <= INT32_MAX;
                                out[j] = (int32_t)x;
                            }
                            *ok = good;
                            return out;
                        },
                        unfit);
}

hipError_t stage_h2d_codes(int32_t* dst, const int32_t* src, size_t n, int32_t n_codes, int device,
                           hipStream_t stream) {
    Stager* st = stager(device, 0);
    if (n < kPackMin || !st || n_codes > 255) return stage_h2d_i32(dst, src, n, device, stream);
    std::unique_lock<std::mutex> g(st->mu);
    if (!packed_ready(st, device)) {
        g.unlock();
        return stage_h2d_i32(dst, src, n, device, stream);
    }
    const size_t per_chunk = kChunk;  // codes: one byte each
    auto encode = [&](char* pin, size_t a0, size_t m, bool*) -> size_t {
        const int32_t* s0 = src + a0;
        uint8_t* o = reinterpret_cast<uint8_t*>(pin);
        st->pool->run(kParts, [&](int i) {
            size_t a, z;
            part_range(m, i, &a, &z);
            for (size_t j = a; j < z; ++j) o[j] = rcp_pack_code8(s0[j], n_codes);
        });
        return m;
    };
    auto land = [&](const char* dev, char* pin, size_t a0, size_t m, size_t bytes, bool, hipStream_t s) {
        hipError_t e = hipMemcpyAsync(const_cast<char*>(dev), pin, bytes, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = rcp_launch_unpack_code8(dev, (int64_t)m, dst + a0, s);
        return e;
    };
    return h2d_packed(st, n, per_chunk, stream, "codes", encode, land);
}

hipError_t stage_h2d_strand(int8_t* dst, const int8_t* src, size_t n, int device, hipStream_t stream) {
    Stager* st = stager(device, 0);
    if (n < kPackMin || !st) return stage_h2d(dst, src, n, device, stream);
    std::unique_lock<std::mutex> g(st->mu);
    if (!ready(st, 0) || !ready_dev(st, device)) {
        g.unlock();
        return stage_h2d(dst, src, n, device, stream);
    }
    const size_t per_chunk = size_t(32) << 20;  // codes (8 MB packed): chunks pipeline encoding and DMA
    auto pack8 = [](uint64_t w) { return rcp_pack_strand8(w); };  // (rcp_pack.h)
    auto encode = [&](char* pin, size_t a0, size_t m, bool*) -> size_t {
        const int8_t* s = src + a0;
        const size_t words = (m + 3) / 4;  // packed bytes
        const size_t groups = m / 8;       // whole groups of eight codes
        st->pool->run(kParts, [&](int i) {
            alignas(16) uint16_t tmp[2048];
            const size_t g0 = groups * (size_t)i / kParts, g1 = groups * (size_t)(i + 1) / kParts;
            for (size_t g = g0; g < g1; g += 2048) {
                const size_t cnt = std::min<size_t>(2048, g1 - g);
                for (size_t q = 0; q < cnt; ++q) {
                    uint64_t w;
                    std::memcpy(&w, s + 8 * (g + q), 8);
                    tmp[q] = (uint16_t)pack8(w);
                }
                copy_nt(pin + 2 * g, reinterpret_cast<const char*>(tmp), 2 * cnt);
            }
        });
        if (m % 8) {  // the last codes
            uint64_t w = 0;
            std::memcpy(&w, s + 8 * groups, m % 8);
            const uint32_t x = pack8(w);
            for (size_t q = 2 * groups; q < words; ++q) pin[q] = (char)(x >> (8 * (q - 2 * groups)));
        }
        return words;
    };
    auto land = [&](const char* dev, char* pin, size_t a0, size_t m, size_t bytes, bool, hipStream_t s) {
        hipError_t e = hipMemcpyAsync(const_cast<char*>(dev), pin, bytes, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = rcp_launch_unpack_strand(dev, (int64_t)m, dst + a0, s);
        return e;
    };
    return h2d_packed(st, n, per_chunk, stream, "strand", encode, land);
}

hipError_t stage_d2h_i32(int32_t* dst, const int32_t* src, size_t n, int device, hipStream_t stream) {
    Stager* st = stager(device, 1);
    if (n < kPackMin || !st) return stage_d2h(dst, src, 4 * n, device, stream);
    std::unique_lock<std::mutex> g(st->mu);
    if (!ready(st, 1) || !ready_dev(st, device)) {
        g.unlock();
        return stage_d2h(dst, src, 4 * n, device, stream);
    }
    const double t1 = trace() ? now_ms() : 0.0;
    const size_t B = (size_t)rcp_pack_block();
    const size_t per_chunk = size_t(16) << 20;  // values: 8 x nb + 2 x per_chunk bytes < the buffers
    const size_t nch = (n + per_chunk - 1) / per_chunk;
    size_t n_raw = 0;
    hipError_t e = hipSuccess;
    // chunk k: packed on the device into dev[k % 2], DMA'd into pin[k % 2]; expanded by the threads
    // one iteration later, while chunk k + 1 is packed and in flight
    auto bytes_of = [&](size_t m) { return 8 * ((m + B - 1) / B) + 2 * m; };
    for (size_t k = 0; k <= nch && e == hipSuccess; ++k) {
        if (k < nch) {
            const int b = (int)(k & 1);
            const size_t a0 = k * per_chunk, m = std::min(per_chunk, n - a0);
            e = rcp_launch_pack_i32(src + a0, (int64_t)m, st->dev[b], stream);
            if (e == hipSuccess) e = hipMemcpyAsync(st->pin[b], st->dev[b], bytes_of(m), hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
        }
        if (k > 0 && e == hipSuccess) {
            const size_t j = k - 1;
            const int b = (int)(j & 1);
            const size_t a0 = j * per_chunk, m = std::min(per_chunk, n - a0), nb = (m + B - 1) / B;
            e = hipEventSynchronize(st->ev[b]);
            if (e != hipSuccess) break;
            const char* pin = st->pin[b];
            const int32_t* base = reinterpret_cast<const int32_t*>(pin);
            const int32_t* flag = base + nb;
            const uint16_t* off = reinterpret_cast<const uint16_t*>(pin + 8 * nb);
            st->pool->run(kParts, [&](int i) {
                alignas(16) int32_t tmp[1024];
                for (size_t bl = nb * (size_t)i / kParts; bl < nb * (size_t)(i + 1) / kParts; ++bl) {
                    if (flag[bl]) continue;  // (copied from the device below)
                    const size_t j0 = bl * B, len = std::min(B, m - j0);
                    const uint32_t bs = (uint32_t)base[bl];
                    for (size_t q = 0; q < len; ++q) tmp[q] = (int32_t)(bs + off[j0 + q]);
                    copy_nt(reinterpret_cast<char*>(dst + a0 + j0), reinterpret_cast<const char*>(tmp), 4 * len);
                }
            });
            // blocks whose values span 2^16 or more: straight from the device array (a chunk with
            // many of them as a whole: one copy)
            size_t raw_here = 0;
            for (size_t bl = 0; bl < nb; ++bl) raw_here += flag[bl] ? 1 : 0;
            n_raw += raw_here;
            // (on the caller's stream, one synchronisation: the next chunk's pack and DMA, already
            // queued, finish first)
            if (raw_here > nb / 32) {
                e = hipMemcpyAsync(dst + a0, src + a0, 4 * m, hipMemcpyDeviceToHost, stream);
            } else {
                for (size_t bl = 0; bl < nb && e == hipSuccess; ++bl) {
                    if (!flag[bl]) continue;
                    const size_t j0 = bl * B, len = std::min(B, m - j0);
                    e = hipMemcpyAsync(dst + a0 + j0, src + a0 + j0, 4 * len, hipMemcpyDeviceToHost, stream);
                }
            }
            if (raw_here && e == hipSuccess) e = hipStreamSynchronize(stream);
        }
    }
    hipError_t e2 = hipEventRecord(st->done, stream);
    if (e2 == hipSuccess) e2 = hipEventSynchronize(st->done);
    if (trace())
        fprintf(stderr, "[stage] d2h-packed i32 %zu values, %zu raw blocks, %.2f ms\n", n, n_raw, now_ms() - t1);
    return e != hipSuccess ? e : e2;
}

hipError_t stage_d2h_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                        int device, hipStream_t stream) {
    if (width == 0 || height == 0) return hipSuccess;
    // the device bytes moved: rows with their padding, except after the last row
    const size_t bytes = spitch * (height - 1) + width;
    Stager* st = stager(device, 1);
    const double t0 = trace() ? now_ms() : 0.0;
    std::unique_lock<std::mutex> g;
    if (bytes >= kDirect && st) g = take(st, bytes);
    const double t1 = trace() ? now_ms() : 0.0;
    if (!g.owns_lock() || !ready(st, 1)) {
        hipError_t e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToHost, stream);
        e = e == hipSuccess ? hipStreamSynchronize(stream) : e;
        if (trace() && bytes >= kDirect)
            fprintf(stderr, "[stage] d2h %zu B direct %.2f ms\n", bytes, now_ms() - t1);
        return e;
    }
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    // device bytes [a, z) of the linear span -> their host rows (padding bytes skipped)
    auto scatter = [&](const char* pin, size_t base, size_t a, size_t z) {
        while (a < z) {
            const size_t row = a / spitch, off = a % spitch;
            if (off >= width) {
                a = (row + 1) * spitch;
                continue;
            }
            const size_t n = std::min(z - a, width - off);
            copy_nt(d + row * dpitch + off, pin + (a - base), n);
            a += n;
        }
    };
    const size_t ch = chunk_of(bytes);
    const size_t nch = (bytes + ch - 1) / ch;
    hipError_t e = hipSuccess;
    for (size_t k = 0; k <= nch && e == hipSuccess; ++k) {
        if (k < nch) {  // DMA chunk k into buffer k % 2 (drained below one iteration ago)
            const int b = (int)(k & 1);
            const size_t a0 = k * ch, len = std::min(ch, bytes - a0);
            e = hipMemcpyAsync(st->pin[b], s + a0, len, hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
        }
        if (k > 0 && e == hipSuccess) {  // drain chunk k - 1 while chunk k is in flight
            const size_t j = k - 1;
            const int b = (int)(j & 1);
            const size_t a0 = j * ch, len = std::min(ch, bytes - a0);
            e = hipEventSynchronize(st->ev[b]);
            if (e != hipSuccess) break;
            const char* pin = st->pin[b];
            st->pool->run(kParts, [&](int i) {
                size_t a, z;
                part_range(len, i, &a, &z);
                if (z > a) scatter(pin, a0, a0 + a, a0 + z);
            });
        }
    }
    hipError_t e2 = hipEventRecord(st->done, stream);
    if (e2 == hipSuccess) e2 = hipEventSynchronize(st->done);
    if (trace()) fprintf(stderr, "[stage] d2h %zu B wait %.2f ms copy %.2f ms\n", bytes, t1 - t0, now_ms() - t1);
    return e != hipSuccess ? e : e2;
}

hipError_t stage_d2h_expand(double* dst, size_t dld, const uint32_t* src, size_t sld, size_t rows, size_t cols,
                            const uint32_t* div, double scale, int device, hipStream_t stream, bool* unavailable) {
    if (unavailable) *unavailable = false;
    if (rows == 0 || cols == 0) return hipSuccess;
    // per row: the reciprocal of a power-of-two width (0 for a NULL row) or the width to divide by
    std::vector<double> rd(rows), dv(rows);
    bool all_pow2 = true;
    for (size_t i = 0; i < rows; ++i) {
        const uint32_t d = div[i];
        const bool p2 = (d & (d - 1)) == 0;
        rd[i] = p2 && d ? 1.0 / (double)d : 0.0;
        dv[i] = p2 ? 0.0 : (double)d;
        all_pow2 = all_pow2 && p2;
    }
    const size_t bytes = 4 * (sld * (cols - 1) + rows);  // device bytes moved (column padding inside)
    Stager* st = stager(device, 1);
    const double t0 = trace() ? now_ms() : 0.0;
    std::unique_lock<std::mutex> g;
    if (st) g = take(st, std::max(bytes, kShared));  // (always the buffers: the expansion needs them)
    const double t1 = trace() ? now_ms() : 0.0;
    if (!g.owns_lock() || !ready(st, 1)) {
        // no pinned buffers on this device (an ordinal past the stagers, or hipHostMalloc refused):
        // the caller downloads the doubles instead
        if (unavailable) *unavailable = true;
        return unavailable ? hipSuccess : hipErrorOutOfMemory;
    }
    // device words [a, z) of the linear span -> their host cells (padding skipped)
    auto scatter = [&](const uint32_t* pin, size_t base, size_t a, size_t z) {
        while (a < z) {
            const size_t col = a / sld, off = a % sld;
            if (off >= rows) {
                a = (col + 1) * sld;
                continue;
            }
            const size_t n = std::min(z - a, rows - off);
            expand_nt(dst + col * dld + off, pin + (a - base), rd.data() + off, dv.data() + off, all_pow2, scale, n);
            a += n;
        }
    };
    const size_t words = bytes / 4;
    hipError_t e = hipSuccess;
    size_t n_raw = 0;
    if (ready_dev(st, device)) {
        // the numerators themselves travel packed: blocks of B words as their minimum + 16-bit
        // offsets (rcp_pack_i32_kernel; C4's are bin sums of a few hundred), a block that does not
        // fit fetched as it is -- 2 bytes a cell over PCIe
        const size_t B = (size_t)rcp_pack_block();
        const size_t per_chunk = size_t(16) << 20;
        const size_t nch = (words + per_chunk - 1) / per_chunk;
        auto bytes_of = [&](size_t m) { return 8 * ((m + B - 1) / B) + 2 * m; };
        std::vector<uint32_t> raw;  // raw blocks of the chunk being drained (host copy)
        std::vector<size_t> raw_blocks;
        for (size_t k = 0; k <= nch && e == hipSuccess; ++k) {
            if (k < nch) {
                const int b = (int)(k & 1);
                const size_t a0 = k * per_chunk, m = std::min(per_chunk, words - a0);
                e = rcp_launch_pack_i32(reinterpret_cast<const int32_t*>(src) + a0, (int64_t)m, st->dev[b], stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(st->pin[b], st->dev[b], bytes_of(m), hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
            }
            if (k > 0 && e == hipSuccess) {
                const size_t j = k - 1;
                const int b = (int)(j & 1);
                const size_t a0 = j * per_chunk, m = std::min(per_chunk, words - a0), nb = (m + B - 1) / B;
                e = hipEventSynchronize(st->ev[b]);
                if (e != hipSuccess) break;
                const char* pin = st->pin[b];
                const int32_t* base = reinterpret_cast<const int32_t*>(pin);
                const int32_t* flag = base + nb;
                const uint16_t* off = reinterpret_cast<const uint16_t*>(pin + 8 * nb);
                // blocks whose values span 2^16 or more come as they are, fetched by THIS thread (on
                // the caller's device and stream; the pool's threads make no HIP calls): a chunk with
                // many of them in one copy, else block by block, all before one synchronisation
                raw_blocks.clear();
                for (size_t bl = 0; bl < nb; ++bl)
                    if (flag[bl]) raw_blocks.push_back(bl);
                n_raw += raw_blocks.size();
                if (!raw_blocks.empty()) {
                    if (raw.size() < m) raw.resize(m);
                    if (raw_blocks.size() > nb / 32) {
                        e = hipMemcpyAsync(raw.data(), src + a0, 4 * m, hipMemcpyDeviceToHost, stream);
                    } else {
                        for (size_t bl : raw_blocks) {
                            const size_t j0 = bl * B, len = std::min(B, m - j0);
                            e = hipMemcpyAsync(raw.data() + j0, src + a0 + j0, 4 * len, hipMemcpyDeviceToHost, stream);
                            if (e != hipSuccess) break;
                        }
                    }
                    if (e == hipSuccess) e = hipStreamSynchronize(stream);
                    if (e != hipSuccess) break;
                }
                const uint32_t* rawp = raw.data();
                st->pool->run(kParts, [&](int i) {
                    uint32_t tmp[1024];
                    for (size_t bl = nb * (size_t)i / kParts; bl < nb * (size_t)(i + 1) / kParts; ++bl) {
                        const size_t j0 = bl * B, len = std::min(B, m - j0);
                        if (flag[bl]) {
                            scatter(rawp + j0, a0 + j0, a0 + j0, a0 + j0 + len);
                            continue;
                        }
                        const uint32_t bs = (uint32_t)base[bl];
                        for (size_t q = 0; q < len; ++q) tmp[q] = bs + off[j0 + q];
                        scatter(tmp, a0 + j0, a0 + j0, a0 + j0 + len);
                    }
                });
            }
        }
    } else {
        const size_t ch = chunk_of(bytes) / 4 / 1024 * 1024;  // words per chunk
        const size_t nch = (words + ch - 1) / ch;
        const char* s = reinterpret_cast<const char*>(src);
        for (size_t k = 0; k <= nch && e == hipSuccess; ++k) {
            if (k < nch) {
                const int b = (int)(k & 1);
                const size_t a0 = k * ch, len = std::min(ch, words - a0);
                e = hipMemcpyAsync(st->pin[b], s + 4 * a0, 4 * len, hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess) e = hipEventRecord(st->ev[b], stream);
            }
            if (k > 0 && e == hipSuccess) {
                const size_t j = k - 1;
                const int b = (int)(j & 1);
                const size_t a0 = j * ch, len = std::min(ch, words - a0);
                e = hipEventSynchronize(st->ev[b]);
                if (e != hipSuccess) break;
                const uint32_t* pin = reinterpret_cast<const uint32_t*>(st->pin[b]);
                st->pool->run(kParts, [&](int i) {
                    const size_t per = (len + kParts - 1) / kParts;
                    const size_t a = std::min(len, per * (size_t)i), z = std::min(len, a + per);
                    if (z > a) scatter(pin, a0, a0 + a, a0 + z);
                });
            }
        }
    }
    hipError_t e2 = hipEventRecord(st->done, stream);
    if (e2 == hipSuccess) e2 = hipEventSynchronize(st->done);
    if (trace())
        fprintf(stderr, "[stage] d2h-expand %zu B (%zu cells, %zu raw blocks) wait %.2f ms copy %.2f ms\n", bytes,
                rows * cols, n_raw, t1 - t0, now_ms() - t1);
    return e != hipSuccess ? e : e2;
}

}  // namespace rcp
