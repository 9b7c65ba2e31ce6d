// rcp_internal.h -- what the host sources of librecoup_amd.so share (not part of the C ABI):
// error reporting, RAII device buffers, the device memory pool, the readset / plan / coverage
// handle layouts and the kernel launchers of rcp_kernels.hip / rcp_rle.hip / rcp_shard.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <functional>
#include <vector>

#include "../../include/recoup_amd.h"
#include "rcp_device.h"

extern "C" {
hipError_t rcp_sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* kin, uint64_t* kout, const int32_t* vin,
                          int32_t* vout, int64_t n, int begin_bit, int end_bit, hipStream_t stream);
hipError_t rcp_launch_unsorted(int64_t n, const uint64_t* keys, uint32_t* flag, hipStream_t stream);
hipError_t rcp_launch_width_end(int64_t n, const int32_t* start, int32_t* width_end, uint32_t* overflow,
                                hipStream_t stream);
hipError_t rcp_launch_order(int64_t n, const int32_t* chrom, const int32_t* start, uint32_t* flag, hipStream_t stream);
hipError_t rcp_launch_expand_runs(int64_t n, int32_t n_runs, const int64_t* run_start, const int32_t* run_value,
                                  int32_t* out, hipStream_t stream);
hipError_t rcp_segmax_scan(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, int64_t n,
                           hipStream_t stream);
hipError_t rcp_launch_locate(const RcpPlanDev* P, hipStream_t stream);
hipError_t rcp_launch_heavy(const RcpPlanDev* P, int grid, hipStream_t stream);
hipError_t rcp_launch_pileup(const RcpPlanDev* P, double* out, int64_t* binsum, int csr, hipStream_t stream);
hipError_t rcp_launch_interp(const RcpPlanDev* P, double* out, hipStream_t stream);
hipError_t rcp_launch_pack(const RcpPlanDev* P, const double* out, uint32_t* q_out, uint32_t* div, uint32_t* bad_row,
                           hipStream_t stream);
hipError_t rcp_launch_gather_rows(const double* out, int64_t ld, const int32_t* rows, int32_t n, int64_t n_cols,
                                  double* dst, hipStream_t stream);
size_t rcp_pileup_lds_bytes(const RcpPlanDev* P, int csr);
size_t rcp_interp_lds_bytes(const RcpPlanDev* P);
int rcp_tile_rows(void);
void rcp_tile_geometry(int* tile, int* rounds_max);
int rcp_lean_max_bins(void);
int rcp_lean_gen_max_bins(void);
size_t rcp_pileup_lean_lds_bytes(const RcpPlanDev* P);
size_t rcp_pileup_rows_lds_bytes(const RcpPlanDev* P);
size_t rcp_pileup_bins_lds_bytes(const RcpPlanDev* P);
int rcp_bins_max_bins(void);
int rcp_bins_min_width(void);
int rcp_rows_window_cap(void);
hipError_t rcp_launch_readset(int64_t n, const int32_t* chrom, const int32_t* start, const int32_t* end,
                              const int8_t* strand, int32_t n_chrom, int32_t strand_filter, int merge, uint64_t* keys,
                              int32_t* vals, hipStream_t stream);
hipError_t rcp_launch_streams(int64_t n, const uint64_t* keys, const int32_t* vals, int64_t* off, int64_t n_off,
                              int2* se, uint64_t* scan_in, hipStream_t stream);
hipError_t rcp_launch_unpack_pmax(int64_t n, const uint64_t* scan_out, int32_t* pmax, hipStream_t stream);
hipError_t rcp_rle_encode_dev(int32_t n_rows, const int64_t* d_off, const int32_t* d_cov, int64_t* d_count,
                              int64_t* d_run_off, void* temp, size_t* temp_bytes, int32_t* d_values,
                              int32_t* d_lengths, int pass, hipStream_t stream);
hipError_t rcp_launch_width_range(int64_t n, const uint64_t* keys, const int32_t* vals, int32_t* mm,
                                  hipStream_t stream);
hipError_t rcp_launch_split_uniform(int64_t n, const int2* se, int32_t* st, int32_t* pmax, hipStream_t stream);
hipError_t rcp_cov_runs_dev(int32_t n_rows, const int64_t* d_off, const int64_t* d_sub_off, int64_t n_sub,
                            const int2* d_sub, const int2* d_rs, const uint8_t* d_valid, int32_t chunk, int64_t* d_cnt,
                            int4* d_info, int64_t* d_base, int64_t* d_run_off, void* temp, size_t* temp_bytes,
                            int32_t* d_values, int32_t* d_lengths, uint32_t* d_bad, int pass, hipStream_t stream);
hipError_t rcp_launch_stream_maxend(int64_t n_streams, const int64_t* off, const int32_t* pmax, int32_t* out,
                                    hipStream_t stream);
hipError_t rcp_launch_dir(int64_t n_entries, int64_t n_streams, const int64_t* dir_off, const int64_t* off,
                          const int32_t* pmax, const int2* se, int shift, int32_t* dir_l, int32_t* dir_u,
                          hipStream_t stream);
hipError_t rcp_launch_dirk(int64_t n_entries, const int32_t* dir_lu, const int32_t* pmax, const int2* se,
                           int32_t* dir_k, hipStream_t stream);
}

namespace rcpi {

// The calling thread's message for rcp_last_error(); returns code.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
extern thread_local std::string g_err;

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(e_ == hipErrorOutOfMemory ? RCP_ENOMEM : RCP_EHIP, "%s: %s (%s:%d)", #expr, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                          \
    } while (0)

// Nothing may escape into the caller's process (an R session): every C++ exception that a
// body can raise (std::bad_alloc from table building, std::system_error from threads) becomes
// an RCP_E* code.
#define RCP_TRY try {
#define RCP_CATCH                                                                         \
    }                                                                                     \
    catch (const std::bad_alloc&) {                                                       \
        return fail(RCP_ENOMEM, "host memory exhausted in %s", __func__);                 \
    }                                                                                     \
    catch (const std::exception& e_) {                                                    \
        return fail(RCP_EINVAL, "%s: %s", __func__, e_.what());                          \
    }                                                                                     \
    catch (...) {                                                                         \
        return fail(RCP_EINVAL, "%s: unexpected C++ exception", __func__);               \
    }

// Device buffer with RAII.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            reset();
            p = o.p;
            bytes = o.bytes;
            o.p = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t alloc(size_t n) {
        reset();
        bytes = n;
        if (n == 0) return hipSuccess;
        return hipMalloc(&p, n);
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// Stream-ordered device memory from the library's caching allocator (rcp_host.cpp): pool_alloc's
// block is usable in stream order on s; pool_free hands it back after the work queued on s so far
hipError_t pool_alloc(void** p, size_t n, hipStream_t s);
void pool_free(void* p, hipStream_t s);

struct PoolBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t s;
    explicit PoolBuf(hipStream_t st) : s(st) {}
    PoolBuf(const PoolBuf&) = delete;
    PoolBuf& operator=(const PoolBuf&) = delete;
    ~PoolBuf() { reset(); }
    void reset() {
        pool_free(p, s);
        p = nullptr;
        bytes = 0;
    }
    hipError_t alloc(size_t n) {
        reset();
        bytes = n;
        if (n == 0) return hipSuccess;
        return pool_alloc(&p, n, s);
    }
    void* release() {  // ownership to the caller
        void* q = p;
        p = nullptr;
        bytes = 0;
        return q;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// Switch to a device for the scope of an API call, restoring the caller's device.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// RCP_OK, or RCP_ENODEVICE / RCP_EINVAL when `dev` is not a visible device
int check_device(int dev);

// Run fn(i) for i in [0, n) on one host thread each (one per GPU), collecting the first failure's
// code and message into the calling thread's rcp_last_error().
template <class F>
int run_per_device(int n, F fn) {
    std::vector<int> rc(n, RCP_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    th.reserve(n);
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            try {
                rc[i] = fn(i);
            } catch (const std::bad_alloc&) {
                rc[i] = fail(RCP_ENOMEM, "host memory exhausted (device thread %d)", i);
            } catch (...) {
                rc[i] = fail(RCP_EINVAL, "unexpected C++ exception (device thread %d)", i);
            }
            if (rc[i]) msg[i] = g_err;  // g_err is thread-local
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[i]) return fail(rc[i], "device %d: %s", i, msg[i].c_str());
    return RCP_OK;
}

// Device rows [src, src + len) of a matrix go to host rows [dst, dst + len)
struct RowRun {
    size_t src, dst, len;
};
// A plan's matrix on the device (column stride plan->out_ld) into a host column-major double
// matrix of column stride host_ld, as bin numerators when the plan allows (rcp_host.cpp); runs
// (NULL: row i to host row i) place the device rows
int download_matrix(rcp_plan* plan, const double* d_out, double* host, size_t host_ld, hipStream_t s,
                    const std::vector<RowRun>* runs = nullptr);
// the numerator download of an R x C column-major device matrix d_out (stride ld): pack(q, div,
// bad_row) fills the numerators, per-row widths and per-row failure marks (zeroed first); rows
// marked come down as doubles apart, or everything does when they are many
int download_packed(const double* d_out, size_t ld, size_t R, size_t C, double scale, double* host, size_t host_ld,
                    int device, hipStream_t s,
                    const std::function<hipError_t(uint32_t* q, uint32_t* div, uint32_t* bad_row)>& pack,
                    const std::vector<RowRun>* runs = nullptr);
// Block [r0, r0 + sub->n_rows) of an n_rows_total-row profile on readset rs: plan, execute, and
// copy its rows of every column into the caller's R column-major matrix `out` (may be NULL) and
// row_valid + r0 (may be NULL); *n_cols receives the plan's column count.  dst_rows (may be NULL):
// the caller's row of each block row instead of r0 + i.  On `stream` (NULL: a stream of its own);
// returns with the copies done (rcp_host.cpp)
int profile_block(const rcp_readset* rs, const rcp_rows_desc* sub, const rcp_bins_desc* bins, double* out,
                  int64_t n_rows_total, int32_t r0, uint8_t* row_valid, int64_t* n_cols, hipStream_t stream = nullptr,
                  const int32_t* dst_rows = nullptr);

// rcp_profile_rle into rows [0, n_rows) of a matrix with column stride out_ld, on stream s
// (rcp_host.cpp)
int profile_rle_impl(const rcp_rle_desc* cov, const rcp_bins_desc* bins, int device, double* out, int64_t out_ld,
                     uint8_t* row_valid, hipStream_t s);

// Contiguous row blocks of near-equal weight from the prefix sums of the row weights (rcp_host.cpp)
std::vector<int32_t> balanced_split(const std::vector<double>& cum, int32_t n_blocks);

// Candidate reads [lo, hi) of every (range, stream slot) of `rows` in the layout of rs the rows
// search (merged for ignore_strand, else strand-split): host [3 * n_seg] (rcp_shard.cpp)
int seg_bounds(const rcp_readset* rs, const rcp_rows_desc* rows, std::vector<uint2>* out);

// Reads [a, b) of a sample as a descriptor of their own (run lists cut to the slice, owned here)
// (rcp_shard.cpp)
struct ReadSlice {
    rcp_reads_desc d{};
    std::vector<int32_t> cv, wv;
    std::vector<int64_t> cl, wl;
};
void slice_reads(const rcp_reads_desc* src, int64_t a, int64_t b, ReadSlice* out);

// rcp_cov_copy of a coverage made of per-device parts (rcp_shard.cpp)
int cov_copy_parts(const rcp_cov* c, int64_t* run_off, int32_t* values, int32_t* lengths, uint8_t* valid);

// A readset with the layouts asked for (rcp_host.cpp): kLayMerged (ignore.strand = TRUE),
// kLayStranded (FALSE); kLayKeep: host input keeps its uploaded copies for a stranded layout
// built at first use; kLayIndexOnly: streams and prefix max only, no bucket directory (a
// readset searched once, never planned on)
// kLayCheckOrder: host input with chromosome runs must be coordinate-sorted (starts ascending
// inside each chromosome's reads): kNotInOrder (> 0, no error message) when it is not
enum { kLayMerged = 1, kLayStranded = 2, kLayKeep = 4, kLayIndexOnly = 8, kLayCheckOrder = 16 };
constexpr int kNotInOrder = 1;
int readset_build(const rcp_reads_desc* d, hipStream_t s, int layouts, rcp_readset** out);

}  // namespace rcpi

// One sorted layout of the reads: streams (chromosome x strand) of start-sorted (start, end)
// pairs with their prefix max of end and bucket directory (rcp_device.h).  A readset keeps two:
// `stranded` (stream c*3 + strand, for findOverlaps with strand compatibility) and `merged`
// (all strands in stream c*3, streams c*3+1, c*3+2 empty: ignore.strand = TRUE, the default),
// so the default path searches and streams one range per segment instead of three.
// A readset's (and a plan's) own arrays, from the same caching allocator (a 4 GB hipMalloc of
// C5's packed reads once took 5.9 s on the box, tools/diag_readset.py), allocated on the build
// stream and handed back after the owner's last work has finished (~rcp_readset: one device
// synchronisation -- what hipFree does implicitly, so a readset destroyed with work still queued
// on it stays safe; ~rcp_plan: its completion event).
namespace rcpi {
struct PoolArr {
    void* p = nullptr;
    size_t bytes = 0;
    PoolArr() = default;
    PoolArr(const PoolArr&) = delete;
    PoolArr& operator=(const PoolArr&) = delete;
    PoolArr(PoolArr&& o) noexcept : p(o.p), bytes(o.bytes) {
        o.p = nullptr;
        o.bytes = 0;
    }
    PoolArr& operator=(PoolArr&& o) noexcept {
        if (this != &o) {
            pool_free(p, nullptr);
            p = o.p;
            bytes = o.bytes;
            o.p = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    ~PoolArr() {
        pool_free(p, nullptr);  // after rcp_readset's device synchronisation
    }
    hipError_t alloc(size_t n, hipStream_t s) {
        if (p) return hipErrorInvalidValue;  // allocated once
        bytes = n;
        if (n == 0) return hipSuccess;
        return pool_alloc(&p, n, s);
    }
    void reset() {
        pool_free(p, nullptr);
        p = nullptr;
        bytes = 0;
    }
    void adopt(PoolBuf& b) {  // a build temporary kept (freed as this array is)
        reset();
        bytes = b.bytes;
        p = b.release();
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct ReadLayout {
    std::vector<int64_t> h_stream_off;  // n_chrom*3 + 1
    std::vector<int64_t> h_dir_off;     // n_chrom*3 + 1
    PoolArr se, pmax, stream_off;
    PoolArr dir_l, dir_off;
    PoolArr dir_k;      // inline-key directory (128 bytes per entry; rcp_device.h)
    int32_t dir_shift = 12;
    PoolArr st;         // the starts alone when every read has one width (st_w = end - start)
    int32_t st_w = 0;
};

}  // namespace rcpi

struct rcp_readset {
    int device = 0;
    int64_t n = 0;  // reads kept (strand filter applied)
    int32_t n_chrom = 0;
    std::vector<int64_t> seqlen;
    rcpi::PoolArr d_seqlen;
    rcpi::ReadLayout stranded, merged;
    bool presorted = false;  // the reads came in (chromosome, start) order (no full radix sort)
    bool has_merged = false; // the merged layout was built (every readset but a strand-split shard's)
    // The stranded layout serves only ignore.strand = FALSE (findOverlaps with strand
    // compatibility); the default TRUE reads the merged one.  Reads uploaded from the host keep
    // their device copies here and the stranded layout is built at its first use
    // (ensure_stranded: a plan with ignore_strand == 0, rcp_readset_info), not by every create.
    std::mutex mu;
    bool stranded_ready = false;
    rcp_reads_desc desc{};  // n, n_chrom, strand_filter of the build
    rcpi::PoolArr keep_chrom, keep_start, keep_end, keep_strand;
    const int32_t *kc = nullptr, *ks = nullptr, *ke = nullptr;
    const int8_t* kst = nullptr;
    // one device synchronisation before the members' arrays go back to the pool (what hipFree
    // does implicitly): work still queued on any stream that reads them has finished
    ~rcp_readset() { (void)hipDeviceSynchronize(); }
};


// the execution state of a plan (rcp_host.cpp)
struct rcp_plan {
    const rcp_readset* rs = nullptr;
    RcpPlanDev dev{};
    int32_t n_rows = 0;
    int64_t n_cols = 0;
    int64_t n_seg = 0;
    std::vector<int64_t> row_len;
    size_t lds = 0;
    int64_t grid = 0;
    int32_t tile_rows = 64;  // rows per pileup workgroup (info)
    // device arrays from the pool, released when the plan's last execution has finished (ev_done,
    // or a device synchronisation when it ran on several streams): no hipMalloc / hipFree -- a
    // device-wide synchronisation -- per plan, which would stall the other threads of a pipeline
    rcpi::PoolArr tables;    // read-only tables
    rcpi::PoolArr work;      // seg_lo / seg_hi / valid / status
    rcpi::PoolArr scratch;   // interpolation scratch
    rcpi::PoolArr rm;        // row-wave kernel: row-major staging of the matrix
    int32_t max_row_len = 0;
    int64_t out_ld = 0;
    uint32_t* status_sets = nullptr;  // 2 x RCP_STATUS_WORDS words in `work`
    int epoch = 1;                    // parity of the last execution (the first one uses set 0)
    // the interpolation rows run on a side stream beside the pileup (fork / join on the caller's
    // stream; made at the first execution that interpolates)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev_done = nullptr;  // recorded after every execution (rcp_host.cpp end_exec)
    hipStream_t last = nullptr;    // the executions' stream, when n_streams == 1
    int n_streams = 0;             // 0, 1, 2 = several
    ~rcp_plan() {  // (on the plan's device: rcp_plan_destroy)
        if (n_streams > 1) (void)hipDeviceSynchronize();
        else if (ev_done) (void)hipEventSynchronize(ev_done);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (side) (void)hipStreamDestroy(side);
    }
};

// a calcCoverage result held on the device (rcp_host.cpp); a coverage of several devices' row
// blocks (rcp_shards_coverage) holds one part per block instead, rows split at `split`
struct rcp_cov {
    int32_t n_rows = 0;
    int64_t n_runs = 0;
    int device = 0;
    rcpi::PoolBuf run_off{nullptr}, values{nullptr}, lengths{nullptr}, valid{nullptr};
    std::vector<std::unique_ptr<rcp_cov>> parts;
    std::vector<int32_t> split;
    std::vector<int32_t> order;  // the parts' rows in the caller's numbering (empty: in order)
    ~rcp_cov() {
        // the buffers go back to the pool after everything queued on the null stream
        run_off.reset();
        values.reset();
        lengths.reset();
        valid.reset();
    }
};
