// rcp_host.cpp -- host side of librecoup_amd.so: the C ABI of include/recoup_amd.h.
//
// Owns device memory (RAII), builds per-plan tables from the reference's semantics and
// launches the gfx950 kernels in rcp_kernels.hip.  Host work is table construction only
// (segment orientation, R-RNG bin layouts, chunking); every per-read / per-base operation
// runs on the GPU.  There is no CPU fallback: without a device every entry point fails with
// RCP_ENODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/recoup_amd.h"
#include "rcp_device.h"
#include "rcp_internal.h"
#include "rcp_rle.h"
#include "rcp_rng.h"
#include "rcp_stage.h"

// auto split off: on one GPU's 1/8, 1/4, 1/2 shard of C4, 4 and 8 column chunks instead of 2
// were slower (1/8: pileup 0.109 -> 0.143 / 0.203 ms; profiles/r02c/lean_chunk_split_ab.log) --
// an item's time is set by its 64 rows' read round trips, not by its width
constexpr int kLeanItemsPerWg = 0;  // work items per persistent workgroup, at least
// Per-base plans (C5's TSS windows: reads piled in the window's middle, so the middle column
// chunks are several times the outer ones' work) on few row tiles -- one GPU's shard -- take at
// least this many work items per workgroup: narrower chunks let the per-XCD claims balance the
// heavy middle items against the light outer ones (with ~1.5 items per workgroup the pass lasts
// as long as the slowest workgroup's heavy items)
constexpr int kLeanItemsPerWgBase = 4;
constexpr int kLeanMinChunkBins = 64;                   // no column chunks narrower than this
constexpr int32_t kFoldConcurrentMaxRows = 8192;        // per-base lean fold of plans in flight, rows at most
// AUTO keeps binned plans of fewer rows on the general kernel: a lean item is 64 rows, the
// general kernel's workgroup 32, and with about one item per workgroup the item's read round
// trips set the pass.  C4 shards (1000 bins of 2 bp), ms per pass lean / general: 25 k rows
// 0.141 / 0.133, 33 k 0.160 / 0.154, 40 k 0.187 / 0.197, 50 k 0.217 / 0.232; per-base C5
// shards stay lean (12.5 k rows: 0.317 / 0.435).  profiles/r03/pipeline/small_shard_kernels.log
constexpr int kLeanMinRowsBinned = 36000;
// Per-base lean plans (baseCoverageMatrix: every part one column per position) take work items
// of two 16-row rounds instead of four: ms per pass four / two rounds, C5 0.752 / 0.673, its
// 1/8 shard 0.272 / 0.253, 1/4 0.319 / 0.290; binned C4 is slower with them (0.553 / 0.563
// pileup; 1/8 shard 0.107 / 0.115).  profiles/r03/pipeline/lean_rounds_ab.log


namespace rcpi {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// The library's device memory: a caching allocator per device.  A readset build's multi-GB sort,
// scan and index buffers cost a hipMalloc / hipFree pair each, and on the box those took 0.3-6 s
// now and then (C5, 500 M reads: a 0.19 s build became 1.4 s and 7.4 s, tools/diag_readset.py);
// a hipMemPool did the same once its size crossed some runtime heuristic (a 1.1 s destroy per
// rep, then a 6 s create: profiles/r05/readset_c5_pool.log).  Here a freed block goes into a free
// list keyed by its size class (8 classes per power of two, so same-sized builds -- repeated
// samples, a streamed sample's row blocks -- get the same blocks back) with an event recorded on
// the stream that freed it; the next allocation of that class on any stream waits for the event
// (stream-ordered, no host synchronisation) and takes the block.  hipMalloc runs only when no
// block of the class is free; device memory goes back to the runtime at rcp_release_pool() or
// when a hipMalloc fails (then every cached block is released and the allocation retried).
namespace {

struct Cached {
    void* p;
    hipEvent_t ev;
};

struct DevCache {
    std::multimap<size_t, Cached> free;  // size class -> block
    std::vector<hipEvent_t> spare;       // recycled events (made on this device)
};

// one lock over every device's lists (allocations are few: a handful per build or plan)
std::mutex g_cache_mu;
std::map<void*, std::pair<int, size_t>> g_live;  // block -> (device, size class)

DevCache& dev_cache(int dev) {
    static DevCache* c = new DevCache[64];  // process lifetime (freed by the OS at exit)
    return c[dev & 63];
}

size_t size_class(size_t n) {
    if (n <= 4096) return 4096;
    const int lg = 63 - __builtin_clzll(n - 1);  // 2^lg < n <= 2^(lg + 1)
    const size_t step = (size_t(1) << lg) / 8;
    return (n + step - 1) / step * step;
}

// return every cached block of the device to the runtime (after its last user's work)
void release_cached(int dev) {
    DevCache& c = dev_cache(dev);
    std::multimap<size_t, Cached> blocks;
    std::vector<hipEvent_t> spare;
    {
        std::lock_guard<std::mutex> lock(g_cache_mu);
        blocks.swap(c.free);
        spare.swap(c.spare);
    }
    DeviceGuard g(dev);
    // (best effort: a failing call here is reported under RCP_TRACE and cleared from the thread's
    // last-error slot, where the next kernel launch's hipGetLastError would find it)
    hipError_t first = hipSuccess;
    const char* what = "";
    auto note = [&](hipError_t e, const char* w) {
        if (e != hipSuccess && first == hipSuccess) {
            first = e;
            what = w;
        }
    };
    for (auto& kv : blocks) {
        if (kv.second.ev) note(hipEventSynchronize(kv.second.ev), "hipEventSynchronize");
        note(hipFree(kv.second.p), "hipFree");
        if (kv.second.ev) note(hipEventDestroy(kv.second.ev), "hipEventDestroy");
    }
    for (hipEvent_t e : spare) note(hipEventDestroy(e), "hipEventDestroy (spare)");
    if (first != hipSuccess) {
        if (rcp::trace_on())
            fprintf(stderr, "[pool] release of %zu blocks: %s: %s\n", blocks.size(), what, hipGetErrorString(first));
        (void)hipGetLastError();
    }
}

}  // namespace

hipError_t pool_alloc(void** p, size_t n, hipStream_t s) {
    *p = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    DevCache& c = dev_cache(dev);
    const size_t cls = size_class(n);
    Cached blk{nullptr, nullptr};
    {
        std::lock_guard<std::mutex> lock(g_cache_mu);
        auto it = c.free.find(cls);
        if (it != c.free.end()) {
            blk = it->second;
            c.free.erase(it);
        }
    }
    if (blk.p) {
        // after the previous user's last work on the block (no event: it was idle when freed)
        e = blk.ev ? hipStreamWaitEvent(s, blk.ev, 0) : hipSuccess;
        std::lock_guard<std::mutex> lock(g_cache_mu);
        if (e != hipSuccess) {
            c.free.emplace(cls, blk);
            return e;
        }
        if (blk.ev) c.spare.push_back(blk.ev);
        g_live[blk.p] = {dev, cls};
        *p = blk.p;
        return hipSuccess;
    }
    e = hipMalloc(p, cls);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        release_cached(dev);
        e = hipMalloc(p, cls);
    }
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    std::lock_guard<std::mutex> lock(g_cache_mu);
    g_live[*p] = {dev, cls};
    return hipSuccess;
}

void pool_free(void* p, hipStream_t s) {
    if (!p) return;
    int dev = 0;
    size_t cls = 0;
    hipEvent_t ev = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_cache_mu);
        auto it = g_live.find(p);
        if (it == g_live.end()) return;  // (not ours)
        dev = it->second.first;
        cls = it->second.second;
        g_live.erase(it);
        DevCache& c = dev_cache(dev);
        if (!c.spare.empty()) {
            ev = c.spare.back();
            c.spare.pop_back();
        }
    }
    DevCache& c = dev_cache(dev);
    DeviceGuard g(dev);  // (s is a stream of the block's device, or the null stream)
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
    if (!ev || hipEventRecord(ev, s) != hipSuccess) {
        // no event: the block goes back only after everything queued on the device so far
        (void)hipDeviceSynchronize();
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
    }
    std::lock_guard<std::mutex> lock(g_cache_mu);
    c.free.emplace(cls, Cached{p, ev});
}

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RCP_ENODEVICE, "no HIP device visible");
    if (dev < 0 || dev >= n) return fail(RCP_EINVAL, "device %d out of range (%d devices)", dev, n);
    return RCP_OK;
}

}  // namespace rcpi
using namespace rcpi;

namespace {

constexpr int kChunkMax = 16384;       // positions of an interpolated slice (block LDS array)
constexpr int kWaveMax = 2047;         // positions per wave sub-chunk (64 x 32 slots incl. the end sentinel)
constexpr int kStageMaxBins = 512;  // bins per chunk (LDS stage = bins x 17 words)
constexpr size_t kLdsBudget = 80 * 1024;  // pileup LDS per workgroup (80 KB: two per CU)
constexpr int kHeavyThreshold = 4096;  // candidate reads per column chunk above which a row is split across workgroups
                                        // (8192 before the lean kernel dealt rows dynamically; C4 0.647 -> 0.633 ms)
constexpr int kDirReads = 8;  // mean reads per directory bucket (the locate kernel's search depth)
constexpr int kHeavySlice = 4096;  // candidate reads per heavy work item
constexpr int kHeavyMaxLen = 16383;    // longer rows never take the heavy path
constexpr int kHeavyGrid = 4096;
// general-kernel plans of at most this many rows search their rows' read ranges in the pileup
// kernel (P.fold): one GPU's share of a region table, where the locate launch and its record round
// trip are a third of the pass
constexpr int kFoldMaxRows = 65536;
// ... and pile a fused-bins chunk of a row with more candidate reads than this with the whole
// workgroup (8 waves, 16 reads per lane in flight) instead of one wave
constexpr int kCoopMin = 8192;
constexpr int kGeneralMaxChunks = 8;  // column chunks a wide binned part is cut into (general kernel)

// A wave's difference array: 64 lanes x per positions (per a power of two >= 4), each lane's
// chunk padded by 4 words (rcp_kernels.hip scan_wave).  Returns the LDS words and the
// position capacity for a chunk of `positions`.
void wave_geometry(int32_t positions, int32_t* words, int32_t* capacity) {
    int32_t need = (positions + 1 + 63) / 64;
    int32_t per = 4;
    while (per < need) per <<= 1;
    *words = 64 * (per + 4);
    *capacity = 64 * per - 1;
}

}  // namespace


// =====================================================================================
// readset
// =====================================================================================
// phase timing of readset builds and plan creation: stderr lines under RCP_TRACE (rcp_stage.h)
struct PlanTimer {
    bool on = rcp::trace_on();
    double t = on ? rcp::trace_ms() : 0.0;
    void mark(const char* what) {
        if (!on) return;
        const double n = rcp::trace_ms();
        fprintf(stderr, "[plan] %-14s %8.3f ms\n", what, n - t);
        t = n;
    }
};
#define PLAN_MARK(what) ptimer.mark(what)
#define LAYOUT_MARK(what) ((void)(ltimer.on && hipStreamSynchronize(s) == hipSuccess), ltimer.mark(what))

int rcp_internal_fail(int code, const char* msg) { return fail(code, "%s", msg); }

extern "C" const char* rcp_version(void) { return "recoup_amd 0.1.0 (gfx950)"; }
extern "C" const char* rcp_last_error(void) { return g_err.c_str(); }

extern "C" int rcp_device_count(int* n) {
    RCP_TRY
    if (!n) return fail(RCP_EINVAL, "n is NULL");
    *n = 0;
    if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
    return RCP_OK;
    RCP_CATCH
}

namespace {

// Sort the reads into layout L (merge = strands share stream c*3) and build its search index.
// `presorted` (in/out): the merged layout, built first, reports whether the reads already came in
// (chromosome, start) order -- a coordinate-sorted BAM's readGAlignments does -- and then skips its
// radix sort; the stranded layout of such reads is a stable sort on the stream id alone (one
// 8-bit pass instead of five: the start order inside each stream is already there).
// Builds one layout of the reads into *L (a fresh ReadLayout: PoolArr allocates once) and
// returns the number of reads it kept in *kept.  Reads rs's seqlengths only.
// directory = false: the search index only (streams, pmax), no bucket directory -- a readset a
// shard build only searches once (rcp_shards_create).
int build_layout(const rcp_readset* rs, const rcp_reads_desc* d, const int32_t* pc, const int32_t* ps,
                 const int32_t* pe, const int8_t* pst, int merge, ReadLayout* L, hipStream_t s, bool* presorted,
                 int64_t* kept_out, bool directory = true) {
    const int64_t n = d->n;
    const int64_t n_streams = (int64_t)d->n_chrom * 3;  // + 1 sentinel stream (dropped reads)
    PlanTimer ltimer;
    PoolBuf keys(s), keys2(s), vals(s), vals2(s), scan_in(s), scan_out(s), temp(s);
    HIP_TRY(keys.alloc(8 * std::max<int64_t>(n, 1)));
    HIP_TRY(keys2.alloc(8 * std::max<int64_t>(n, 1)));
    HIP_TRY(vals.alloc(4 * std::max<int64_t>(n, 1)));
    HIP_TRY(vals2.alloc(4 * std::max<int64_t>(n, 1)));
    HIP_TRY(rcp_launch_readset(n, pc, ps, pe, pst, d->n_chrom, d->strand_filter, merge, keys.as<uint64_t>(),
                               vals.as<int32_t>(), s));
    LAYOUT_MARK("  keys");
    int end_bit = 32;
    while ((int64_t(1) << (end_bit - 32)) <= n_streams) ++end_bit;
    bool sorted_in = false;
    if (merge && n > 1) {
        // keys are (stream, start): non-decreasing <=> (chromosome, start) order, no dropped read
        // (the sentinel stream) before a kept one
        PoolBuf flag(s);
        HIP_TRY(flag.alloc(4));
        HIP_TRY(hipMemsetAsync(flag.p, 0, 4, s));
        HIP_TRY(rcp_launch_unsorted(n, keys.as<uint64_t>(), flag.as<uint32_t>(), s));
        uint32_t h = 1;
        HIP_TRY(hipMemcpyAsync(&h, flag.p, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        sorted_in = h == 0;
        *presorted = sorted_in;
    }
    const int begin_bit = (!merge && *presorted) ? 32 : 0;
    size_t tb = 0;
    if (n > 0 && !sorted_in) {
        HIP_TRY(rcp_sort_pairs(nullptr, &tb, keys.as<uint64_t>(), keys2.as<uint64_t>(), vals.as<int32_t>(),
                               vals2.as<int32_t>(), n, begin_bit, end_bit, s));
        HIP_TRY(temp.alloc(tb));
        HIP_TRY(rcp_sort_pairs(temp.p, &tb, keys.as<uint64_t>(), keys2.as<uint64_t>(), vals.as<int32_t>(),
                               vals2.as<int32_t>(), n, begin_bit, end_bit, s));
    }
    LAYOUT_MARK("  sort");
    if (sorted_in) {
        std::swap(keys.p, keys2.p);
        std::swap(keys.bytes, keys2.bytes);
        std::swap(vals.p, vals2.p);
        std::swap(vals.bytes, vals2.bytes);
    }
    keys.reset();
    vals.reset();
    // reads of one width (fixed read lengths, fragments extended to fragLen): their ends ascend
    // with the starts inside a stream, so pmax = end (no segmented scan) and the pileup
    // kernels stream the starts alone (half their read bytes)
    bool uniform = false;
    if (n > 0) {
        PoolBuf mm(s);
        HIP_TRY(mm.alloc(8));
        const int32_t seed[2] = {INT32_MAX, INT32_MIN};
        HIP_TRY(hipMemcpyAsync(mm.p, seed, 8, hipMemcpyHostToDevice, s));
        HIP_TRY(rcp_launch_width_range(n, keys2.as<uint64_t>(), vals2.as<int32_t>(), mm.as<int32_t>(), s));
        int32_t h_mm[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(h_mm, mm.p, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        uniform = h_mm[0] == h_mm[1] && h_mm[0] >= 0;
        if (uniform) L->st_w = h_mm[0];
    }
    LAYOUT_MARK("  width range");
    HIP_TRY(L->stream_off.alloc(8 * (n_streams + 2), s));
    HIP_TRY(L->se.alloc(8 * std::max<int64_t>(n, 1), s));
    if (!uniform) HIP_TRY(scan_in.alloc(8 * std::max<int64_t>(n, 1)));
    HIP_TRY(rcp_launch_streams(n, keys2.as<uint64_t>(), vals2.as<int32_t>(), L->stream_off.as<int64_t>(),
                               n_streams + 2, L->se.as<int2>(), uniform ? nullptr : scan_in.as<uint64_t>(), s));
    LAYOUT_MARK("  streams+pack");
    keys2.reset();
    vals2.reset();
    HIP_TRY(L->pmax.alloc(4 * std::max<int64_t>(n, 1), s));
    if (uniform) {
        HIP_TRY(L->st.alloc(4 * (size_t)n, s));
        HIP_TRY(rcp_launch_split_uniform(n, L->se.as<int2>(), L->st.as<int32_t>(), L->pmax.as<int32_t>(), s));
    } else {
        HIP_TRY(scan_out.alloc(8 * std::max<int64_t>(n, 1)));
        if (n > 0) {
            size_t tb2 = 0;
            HIP_TRY(rcp_segmax_scan(nullptr, &tb2, scan_in.as<uint64_t>(), scan_out.as<uint64_t>(), n, s));
            if (tb2 > temp.bytes) HIP_TRY(temp.alloc(tb2));
            HIP_TRY(rcp_segmax_scan(temp.p, &tb2, scan_in.as<uint64_t>(), scan_out.as<uint64_t>(), n, s));
        }
        HIP_TRY(rcp_launch_unpack_pmax(n, scan_out.as<uint64_t>(), L->pmax.as<int32_t>(), s));
    }
    LAYOUT_MARK("  pmax");
    scan_in.reset();
    scan_out.reset();
    temp.reset();
    LAYOUT_MARK("  frees");
    L->h_stream_off.resize(n_streams + 2);
    HIP_TRY(hipMemcpyAsync(L->h_stream_off.data(), L->stream_off.p, 8 * (n_streams + 2), hipMemcpyDeviceToHost, s));
    if (!directory) {
        HIP_TRY(hipStreamSynchronize(s));
        *kept_out = L->h_stream_off[n_streams];
        L->h_stream_off.resize(n_streams + 1);
        return RCP_OK;
    }
    // ---- bucket directory: ~32 reads of a stream per bucket on average
    PoolBuf maxend(s);
    HIP_TRY(maxend.alloc(4 * std::max<int64_t>(n_streams, 1)));
    HIP_TRY(rcp_launch_stream_maxend(n_streams, L->stream_off.as<int64_t>(), L->pmax.as<int32_t>(),
                                     maxend.as<int32_t>(), s));
    std::vector<int32_t> h_maxend(std::max<int64_t>(n_streams, 1));
    HIP_TRY(hipMemcpyAsync(h_maxend.data(), maxend.p, 4 * n_streams, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int64_t kept = L->h_stream_off[n_streams];
    L->h_stream_off.resize(n_streams + 1);
    std::vector<int64_t> span(d->n_chrom, 0);
    double genome = 0;
    for (int c = 0; c < d->n_chrom; ++c) {
        int64_t m = std::max<int64_t>(rs->seqlen[c], 0);
        for (int st = 0; st < 3; ++st) m = std::max<int64_t>(m, h_maxend[c * 3 + st]);
        span[c] = m;
        genome += (double)m;
    }
    const int used = merge ? 1 : 3;  // streams per chromosome that hold reads
    const double want = kept > 0 ? (double)kDirReads * used * genome / (double)kept : 1e9;
    int shift = 6;
    while (shift < 24 && (double)(int64_t(1) << (shift + 1)) <= want) ++shift;
    L->dir_shift = shift;
    std::vector<int64_t> doff(n_streams + 1, 0);
    for (int c = 0; c < d->n_chrom; ++c) {
        for (int st = 0; st < 3; ++st) {
            // buckets 0 .. nb-1, entries 0 .. nb (an empty stream gets one bucket)
            const int64_t nb = (merge && st > 0) ? 1 : (span[c] >> shift) + 1;
            doff[c * 3 + st + 1] = doff[c * 3 + st] + nb + 1;
        }
    }
    const int64_t ne = doff[n_streams];
    HIP_TRY(L->dir_off.alloc(8 * (n_streams + 1), s));
    HIP_TRY(L->dir_l.alloc(8 * std::max<int64_t>(ne, 1), s));  // interleaved (l, u) per entry
    HIP_TRY(hipMemcpyAsync(L->dir_off.p, doff.data(), 8 * (n_streams + 1), hipMemcpyHostToDevice, s));
    L->h_dir_off = doff;
    HIP_TRY(rcp_launch_dir(ne, n_streams, L->dir_off.as<int64_t>(), L->stream_off.as<int64_t>(),
                           L->pmax.as<int32_t>(), L->se.as<int2>(), shift, L->dir_l.as<int32_t>(),
                           L->dir_l.as<int32_t>() + 1, s));
    HIP_TRY(L->dir_k.alloc(128 * std::max<int64_t>(ne, 1), s));
    HIP_TRY(rcp_launch_dirk(ne, L->dir_l.as<int32_t>(), L->pmax.as<int32_t>(), L->se.as<int2>(),
                            L->dir_k.as<int32_t>(), s));
    HIP_TRY(hipStreamSynchronize(s));
    LAYOUT_MARK("  directory");
    *kept_out = kept;
    return RCP_OK;
}

}  // namespace

namespace {

// The stranded layout of a readset whose reads were uploaded from the host, built once at its
// first use from the kept device copies (which are then released).
int ensure_stranded(const rcp_readset* crs) {
    rcp_readset* rs = const_cast<rcp_readset*>(crs);
    std::lock_guard<std::mutex> lock(rs->mu);
    if (rs->stranded_ready) return RCP_OK;
    if (!rs->kc && !rs->ks) return fail(RCP_EINVAL, "this readset holds no strand-split layout (a shard built for ignore.strand = TRUE)");
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);
    bool presorted = rs->presorted;
    int64_t kept = 0;
    // built into a local layout, moved in only when complete: a failed build (e.g. out of
    // memory) leaves no half-allocated arrays behind, so a later call can build it again
    ReadLayout L;
    const int rc = build_layout(rs, &rs->desc, rs->kc, rs->ks, rs->ke, rs->kst, 0, &L, nullptr, &presorted, &kept);
    if (rc) return rc;
    if (kept != rs->n) return fail(RCP_EINVAL, "internal: stranded layout kept %lld reads, merged %lld",
                                   (long long)kept, (long long)rs->n);
    rs->stranded = std::move(L);
    rs->keep_chrom.reset();
    rs->keep_start.reset();
    rs->keep_end.reset();
    rs->keep_strand.reset();
    rs->kc = rs->ks = rs->ke = nullptr;
    rs->kst = nullptr;
    rs->stranded_ready = true;
    return RCP_OK;
}

}  // namespace

namespace rcpi {

// the second H2D lane's stream of a device (rcp_readset_create), made on first use
constexpr int64_t kTwoLaneMin = int64_t(1) << 22;  // reads; fewer go up on one lane
static hipStream_t lane_stream(int device) {
    static std::mutex mu;
    static hipStream_t st[64] = {};
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!st[device]) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) cur = -1;
        if ((cur == device || hipSetDevice(device) == hipSuccess) &&
            hipStreamCreateWithFlags(&st[device], hipStreamNonBlocking) != hipSuccess)
            st[device] = nullptr;
        (void)hipGetLastError();
        if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
    }
    return st[device];
}

// The read descriptor's shape (sizes, NULL arrays, runs that cover the reads), before any copy:
// what readset_build and every entry point taking host read arrays check first
int validate_reads(const rcp_reads_desc* d) {
    if (d->n < 0 || d->n >= (int64_t(1) << 31)) return fail(RCP_EUNSUPPORTED, "read count %lld outside [0, 2^31)", (long long)d->n);
    if (d->n_chrom <= 0 || d->n_chrom > (1 << 20)) return fail(RCP_EINVAL, "n_chrom = %d", d->n_chrom);
    if (d->n > 0 && (!d->start || !d->strand)) return fail(RCP_EINVAL, "NULL read array");
    if (d->n > 0 && !d->chrom) {
        if (d->n_chrom_runs <= 0 || !d->chrom_run_value || !d->chrom_run_length)
            return fail(RCP_EINVAL, "chrom is NULL and no chromosome runs are given");
        int64_t tot = 0;
        for (int32_t k = 0; k < d->n_chrom_runs; ++k) {
            if (d->chrom_run_length[k] <= 0) return fail(RCP_EINVAL, "chromosome run %d has length %lld", k,
                                                         (long long)d->chrom_run_length[k]);
            tot += d->chrom_run_length[k];
        }
        if (tot != d->n) return fail(RCP_EINVAL, "chromosome runs cover %lld reads, not %lld", (long long)tot,
                                     (long long)d->n);
    }
    if (d->n > 0 && !d->end) {
        if (d->n_width_runs <= 0 || !d->width_run_value || !d->width_run_length)
            return fail(RCP_EINVAL, "end is NULL and no width runs are given");
        int64_t tot = 0;
        for (int32_t k = 0; k < d->n_width_runs; ++k) {
            if (d->width_run_length[k] <= 0) return fail(RCP_EINVAL, "width run %d has length %lld", k,
                                                         (long long)d->width_run_length[k]);
            if (d->width_run_value[k] < 0) return fail(RCP_EINVAL, "width run %d has width %d", k, d->width_run_value[k]);
            tot += d->width_run_length[k];
        }
        if (tot != d->n) return fail(RCP_EINVAL, "width runs cover %lld reads, not %lld", (long long)tot,
                                     (long long)d->n);
    }
    if (d->strand_filter < -1 || d->strand_filter > 2) return fail(RCP_EINVAL, "strand_filter = %d", d->strand_filter);
    return RCP_OK;
}

// A row table's shape: non-NULL arrays, seg_off from 0 and never decreasing
int validate_rows(const rcp_rows_desc* rows) {
    const int32_t R = rows->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && (!rows->seg_off || !rows->seg_chrom || !rows->seg_start || !rows->seg_end || !rows->seg_strand))
        return fail(RCP_EINVAL, "NULL row array");
    if (R > 0 && rows->seg_off[0] != 0) return fail(RCP_EINVAL, "seg_off[0] != 0");
    for (int32_t r = 0; r < R; ++r)
        if (rows->seg_off[r + 1] < rows->seg_off[r]) return fail(RCP_EINVAL, "seg_off not monotone at row %d", r);
    return RCP_OK;
}

int readset_build(const rcp_reads_desc* d, hipStream_t s, int layouts, rcp_readset** out) {
    if (!d || !out) return fail(RCP_EINVAL, "NULL argument");
    if (!(layouts & (kLayMerged | kLayStranded))) return fail(RCP_EINVAL, "internal: no layout requested");
    *out = nullptr;
    int rc = check_device(d->device);
    if (rc) return rc;
    rc = validate_reads(d);
    if (rc) return rc;
    DeviceGuard g(d->device);
    HIP_TRY(g.err);
    auto rs = std::make_unique<rcp_readset>();
    rs->device = d->device;
    rs->n_chrom = d->n_chrom;
    rs->seqlen.assign(d->n_chrom, -1);
    if (d->seqlen)
        for (int c = 0; c < d->n_chrom; ++c) rs->seqlen[c] = d->seqlen[c] < 0 ? -1 : d->seqlen[c];
    const int64_t n = d->n;
    PlanTimer ptimer;

    // inputs on device
    PoolBuf in_chrom(s), in_start(s), in_end(s), in_strand(s), runs(s), wruns(s);
    const int32_t *pc = d->chrom, *ps = d->start, *pe = d->end;
    const int8_t* pst = d->strand;
    if (!d->chrom && n > 0) {
        // seqnames as runs: expanded on the device (never crosses PCIe)
        std::vector<int64_t> rstart(d->n_chrom_runs + 1, 0);
        for (int32_t k = 0; k < d->n_chrom_runs; ++k) rstart[k + 1] = rstart[k] + d->chrom_run_length[k];
        HIP_TRY(runs.alloc(8 * rstart.size() + 4 * (size_t)d->n_chrom_runs));
        HIP_TRY(hipMemcpyAsync(runs.p, rstart.data(), 8 * rstart.size(), hipMemcpyHostToDevice, s));
        int32_t* rv = reinterpret_cast<int32_t*>(runs.as<char>() + 8 * rstart.size());
        HIP_TRY(hipMemcpyAsync(rv, d->chrom_run_value, 4 * (size_t)d->n_chrom_runs, hipMemcpyHostToDevice, s));
        HIP_TRY(in_chrom.alloc(4 * n));
        HIP_TRY(rcp_launch_expand_runs(n, d->n_chrom_runs, runs.as<int64_t>(), rv, in_chrom.as<int32_t>(), s));
        HIP_TRY(hipStreamSynchronize(s));  // rstart is released on return
        pc = in_chrom.as<int32_t>();
    }
    if (!d->on_device && n > 0) {
        if (d->chrom) HIP_TRY(in_chrom.alloc(4 * n));
        HIP_TRY(in_start.alloc(4 * n));
        if (d->end) HIP_TRY(in_end.alloc(4 * n));
        HIP_TRY(in_strand.alloc(n));
        // caller-owned pageable arrays (R vectors): pinned double-buffered staging (rcp_stage.h),
        // coordinates as 16-bit offsets within blocks and strands four to a byte where they fit.
        // With one chromosome code per read (unsorted reads: R hands over per-read codes), the
        // codes and strands -- host-encoded, their time is the copy threads' -- go up through the
        // second H2D lane on a second thread and stream while this thread sends the starts and
        // ends, whose time is the DMA's (RCP_ONE_H2D_LANE: diagnostics A/B, one lane)
        hipStream_t s2 = d->chrom && n >= kTwoLaneMin && !std::getenv("RCP_ONE_H2D_LANE") ? lane_stream(d->device) : nullptr;
        hipEvent_t ready_ev = nullptr;
        if (s2) {
            // s2 after the allocations' stream-ordered waits on s
            if (hipEventCreateWithFlags(&ready_ev, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ready_ev, s) != hipSuccess || hipStreamWaitEvent(s2, ready_ev, 0) != hipSuccess) {
                (void)hipGetLastError();
                if (ready_ev) (void)hipEventDestroy(ready_ev);
                ready_ev = nullptr;
                s2 = nullptr;
            }
        }
        hipError_t lane_err = hipSuccess;
        std::thread lane1;
        struct Join {  // joined on every way out, exceptions included
            std::thread& t;
            ~Join() {
                if (t.joinable()) t.join();
            }
        } join_lane1{lane1};
        if (s2) {
            lane1 = std::thread([&] {
                try {
                    lane_err = hipSetDevice(d->device);
                    rcp::H2dLane lane(1);
                    if (lane_err == hipSuccess)
                        lane_err = rcp::stage_h2d_codes(in_chrom.as<int32_t>(), d->chrom, (size_t)n, d->n_chrom, d->device, s2);
                    if (lane_err == hipSuccess)
                        lane_err = rcp::stage_h2d_strand(in_strand.as<int8_t>(), d->strand, (size_t)n, d->device, s2);
                } catch (...) {
                    lane_err = hipErrorOutOfMemory;  // (a host allocation of the staging failed)
                }
            });
        }
        bool widths = false;
        // (the lane-1 thread is joined before any return)
        auto lane0 = [&]() -> hipError_t {
            hipError_t e = hipSuccess;
            if (d->chrom && !s2) e = rcp::stage_h2d_codes(in_chrom.as<int32_t>(), d->chrom, (size_t)n, d->n_chrom, d->device, s);
            if (e == hipSuccess) e = rcp::stage_h2d_i32(in_start.as<int32_t>(), d->start, (size_t)n, d->device, s);
            // ends go up as widths (a block of them spans < 2^16 whatever the reads' order: 2 bytes
            // a read where unsorted ends go raw) and are formed again on the device
            if (e == hipSuccess && d->end) {
                bool unfit = false;
                e = rcp::stage_h2d_width(in_end.as<int32_t>(), d->start, d->end, (size_t)n, d->device, s, &unfit);
                if (e == hipSuccess && unfit) e = rcp::stage_h2d_i32(in_end.as<int32_t>(), d->end, (size_t)n, d->device, s);
                widths = !unfit;
            }
            if (e == hipSuccess && !s2) e = rcp::stage_h2d_strand(in_strand.as<int8_t>(), d->strand, (size_t)n, d->device, s);
            return e;
        };
        const hipError_t e0 = lane0();
        if (lane1.joinable()) lane1.join();
        if (ready_ev) (void)hipEventDestroy(ready_ev);
        HIP_TRY(e0);
        HIP_TRY(lane_err);
        pc = in_chrom.as<int32_t>();
        ps = in_start.as<int32_t>();
        if (d->end) pe = in_end.as<int32_t>();
        pst = in_strand.as<int8_t>();
        if (widths) {
            PoolBuf over(s);
            HIP_TRY(over.alloc(4));
            HIP_TRY(hipMemsetAsync(over.p, 0, 4, s));
            HIP_TRY(rcp_launch_width_end(n, ps, in_end.as<int32_t>(), over.as<uint32_t>(), s));
            uint32_t h_over = 0;
            HIP_TRY(hipMemcpyAsync(&h_over, over.p, 4, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (h_over) return fail(RCP_EINVAL, "internal: a read's end formed from its width overflows");
        }
    }
    if (!d->end && n > 0) {
        // widths as runs: expanded on the device, end = start + width - 1 formed there
        std::vector<int64_t> rstart(d->n_width_runs + 1, 0);
        for (int32_t k = 0; k < d->n_width_runs; ++k) rstart[k + 1] = rstart[k] + d->width_run_length[k];
        HIP_TRY(wruns.alloc(8 * rstart.size() + 4 * (size_t)d->n_width_runs + 4));
        HIP_TRY(hipMemcpyAsync(wruns.p, rstart.data(), 8 * rstart.size(), hipMemcpyHostToDevice, s));
        int32_t* wv = reinterpret_cast<int32_t*>(wruns.as<char>() + 8 * rstart.size());
        uint32_t* overflow = reinterpret_cast<uint32_t*>(wv + d->n_width_runs);
        HIP_TRY(hipMemcpyAsync(wv, d->width_run_value, 4 * (size_t)d->n_width_runs, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(overflow, 0, 4, s));
        HIP_TRY(in_end.alloc(4 * n));
        HIP_TRY(rcp_launch_expand_runs(n, d->n_width_runs, wruns.as<int64_t>(), wv, in_end.as<int32_t>(), s));
        HIP_TRY(rcp_launch_width_end(n, ps, in_end.as<int32_t>(), overflow, s));
        uint32_t h_over = 0;
        HIP_TRY(hipMemcpyAsync(&h_over, overflow, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));  // rstart is released on return
        if (h_over) return fail(RCP_EUNSUPPORTED, "a read's start + width - 1 exceeds 2^31 - 1");
        pe = in_end.as<int32_t>();
    }
    if ((layouts & kLayCheckOrder) && n > 1) {
        PoolBuf flag(s);
        HIP_TRY(flag.alloc(4));
        HIP_TRY(hipMemsetAsync(flag.p, 0, 4, s));
        HIP_TRY(rcp_launch_order(n, pc, ps, flag.as<uint32_t>(), s));
        uint32_t h_flag = 0;
        HIP_TRY(hipMemcpyAsync(&h_flag, flag.p, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (h_flag) return kNotInOrder;
    }
    PLAN_MARK("reads H2D");
    bool presorted = false;
    int64_t kept = 0;
    const bool dir = !(layouts & kLayIndexOnly);
    if (layouts & kLayMerged) {
        rc = build_layout(rs.get(), d, pc, ps, pe, pst, 1, &rs->merged, s, &presorted, &kept, dir);
        if (rc) return rc;
        rs->n = kept;
        rs->has_merged = true;
        PLAN_MARK("merged layout");
    }
    rs->presorted = presorted;
    rs->desc = *d;
    if (layouts & kLayStranded) {
        int64_t kept2 = 0;
        rc = build_layout(rs.get(), d, pc, ps, pe, pst, 0, &rs->stranded, s, &presorted, &kept2, dir);
        if (rc) return rc;
        if ((layouts & kLayMerged) && kept2 != kept)
            return fail(RCP_EINVAL, "internal: stranded layout kept %lld reads, merged %lld", (long long)kept2,
                        (long long)kept);
        rs->n = kept2;
        rs->stranded_ready = true;
        PLAN_MARK("stranded layout");
    } else if (!d->on_device && (layouts & kLayKeep)) {
        // keep the uploaded copies for a later stranded layout (ensure_stranded)
        rs->keep_chrom.adopt(in_chrom);
        rs->keep_start.adopt(in_start);
        rs->keep_end.adopt(in_end);
        rs->keep_strand.adopt(in_strand);
        rs->kc = pc;
        rs->ks = ps;
        rs->ke = pe;
        rs->kst = pst;
    }
    HIP_TRY(rs->d_seqlen.alloc(8 * d->n_chrom, s));
    HIP_TRY(hipMemcpyAsync(rs->d_seqlen.p, rs->seqlen.data(), 8 * d->n_chrom, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out = rs.release();
    return RCP_OK;
}

}  // namespace rcpi

extern "C" int rcp_readset_create(const rcp_reads_desc* d, void* hip_stream, rcp_readset** out) {
    RCP_TRY
    if (!d) return fail(RCP_EINVAL, "NULL argument");
    // device arrays are the caller's (not ours to keep): both layouts now; host arrays: the
    // merged layout, the uploaded copies kept for the stranded one at its first use
    const int layouts = d->on_device ? (kLayMerged | kLayStranded) : (kLayMerged | kLayKeep);
    return readset_build(d, static_cast<hipStream_t>(hip_stream), layouts, out);
    RCP_CATCH
}

extern "C" int rcp_readset_destroy(rcp_readset* rs) {
    RCP_TRY
    if (!rs) return RCP_OK;
    DeviceGuard g(rs->device);
    delete rs;
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_release_pool(int device) {
    RCP_TRY
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    HIP_TRY(g.err);
    release_cached(device);
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_readset_info(const rcp_readset* rs, int64_t* n_reads, int64_t* stream_off) {
    RCP_TRY
    if (!rs) return fail(RCP_EINVAL, "NULL readset");
    if (n_reads) *n_reads = rs->n;
    if (stream_off) {
        const int rc = ensure_stranded(rs);
        if (rc) return rc;
        std::memcpy(stream_off, rs->stranded.h_stream_off.data(), 8 * rs->stranded.h_stream_off.size());
    }
    return RCP_OK;
    RCP_CATCH
}

// =====================================================================================
// plan
// =====================================================================================

namespace {

// A new execution: alternate the status sets (RcpPlanDev::status / status_prev); the locate
// kernel clears the previous execution's heavy slots and zeroes its set.
// after an execution's launches on s: the plan's arrays stay allocated until this point (rcp_plan)
int end_exec(rcp_plan* plan, hipStream_t s) {
    if (plan->n_streams == 0) {
        plan->last = s;
        plan->n_streams = 1;
    } else if (plan->last != s) {
        plan->n_streams = 2;
    }
    if (!plan->ev_done) HIP_TRY(hipEventCreateWithFlags(&plan->ev_done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(plan->ev_done, s));
    return RCP_OK;
}

void begin_exec(rcp_plan* plan) {
    plan->epoch ^= 1;
    plan->dev.status = plan->status_sets + RCP_STATUS_WORDS * plan->epoch;
    plan->dev.status_prev = plan->status_sets + RCP_STATUS_WORDS * (plan->epoch ^ 1);
}

struct Builder {
    // host copies of the device tables
    std::vector<int32_t> row_chrom, row_seg, row_len;
    std::vector<uint8_t> row_static;
    std::vector<RcpSeg> segs;
    std::vector<int32_t> lay_index, lay_cnt;
    std::vector<std::pair<int32_t, int32_t>> lay_regions;  // (offset in lay_cnt, n bins)
    std::vector<int32_t> interp_row, interp_part, interp_mode, interp_pos, nb_pos;
};

uint8_t stream_mask(int ignore_strand, int8_t q) {
    // findOverlaps strand compatibility: '*' matches everything (Appendix A, Q2)
    if (ignore_strand) return 0x1;  // the merged layout: every strand in stream 0
    if (q == RCP_STRAND_ANY) return 0x7;
    return (uint8_t)((1u << q) | (1u << RCP_STRAND_ANY));
}

int build_rows(const rcp_readset* rs, const rcp_rows_desc* rows, Builder* B) {
    const int R = rows->n_rows;
    B->row_chrom.assign(R, -1);
    B->row_seg.assign(R + 1, 0);
    B->row_len.assign(R, 0);
    B->row_static.assign(R, 0);
    for (int r = 0; r < R; ++r) {
        const int64_t j0 = rows->seg_off[r], j1 = rows->seg_off[r + 1];
        if (j1 < j0) return fail(RCP_EINVAL, "seg_off not monotone at row %d", r);
        B->row_seg[r] = (int32_t)B->segs.size();
        if (j1 == j0) {
            B->row_static[r] = 1;
            continue;
        }
        const int32_t chrom = rows->seg_chrom[j0];
        B->row_chrom[r] = chrom;
        if (chrom < 0 || chrom >= rs->n_chrom) B->row_static[r] = 1;
        int32_t off = 0;
        // groups appear as contiguous runs of seg_group
        int64_t g0 = j0;
        int prev_group = -1;
        while (g0 < j1) {
            const int grp = rows->seg_group ? rows->seg_group[g0] : 0;
            if (grp < 0 || grp > 3) return fail(RCP_EINVAL, "seg_group %d outside 0..3 (row %d)", grp, r);
            if (grp <= prev_group) return fail(RCP_EINVAL, "groups of row %d not contiguous/increasing", r);
            prev_group = grp;
            int64_t g1 = g0;
            while (g1 < j1 && (rows->seg_group ? rows->seg_group[g1] : 0) == grp) ++g1;
            const bool multi = rows->group_is_list && rows->group_is_list[grp];
            const bool rev_group = rows->seg_strand[g0] == RCP_STRAND_MINUS;  // strand(x)[1] == "-"
            const int32_t gfirst = (int32_t)B->segs.size();
            const int32_t gcount = (int32_t)(g1 - g0);
            if (gcount > 32767) return fail(RCP_EUNSUPPORTED, "more than 32767 ranges in one mask element");
            for (int64_t q = 0; q < gcount; ++q) {
                const int64_t j = rev_group ? (g1 - 1 - q) : (g0 + q);
                if (rows->seg_chrom[j] != chrom) {
                    if (multi) return fail(RCP_EUNSUPPORTED, "row %d: mask element spans several chromosomes", r);
                    return fail(RCP_EUNSUPPORTED, "row %d: groups on different chromosomes", r);
                }
                const int32_t s = rows->seg_start[j], e = rows->seg_end[j];
                RcpSeg sg{};
                sg.gfirst = gfirst;
                sg.gcount = (int16_t)gcount;
                sg.multi = multi ? 1 : 0;
                sg.group = (uint8_t)grp;
                sg.streams = stream_mask(rows->ignore_strand, rows->seg_strand[j]);
                if (e >= s) {
                    // i2k piece s:e; R drops index 0 and fails on negative indices
                    if (s < 0) B->row_static[r] = 1;
                    sg.lo = std::max<int32_t>(s, 1);
                    sg.hi = e;
                    sg.query_ok = 1;
                    sg.rev = rev_group ? 1 : 0;
                    if (sg.hi < sg.lo) continue;  // only index 0: nothing left
                } else {
                    // zero-width range: findOverlaps finds nothing (documented); s:(s-1) still
                    // yields two positions, which only matters for rows that are NULL anyway
                    if (multi) return fail(RCP_EUNSUPPORTED, "row %d: zero-width range inside a range list", r);
                    if (e < 0) B->row_static[r] = 1;
                    sg.lo = std::max<int32_t>(e, 1);
                    sg.hi = s;
                    sg.query_ok = 0;
                    sg.rev = rev_group ? 0 : 1;
                    if (sg.hi < sg.lo) continue;
                }
                sg.off = off;
                off += sg.hi - sg.lo + 1;
                B->segs.push_back(sg);
            }
            // fix gcount for skipped empty pieces
            const int32_t kept = (int32_t)B->segs.size() - gfirst;
            for (int32_t q = gfirst; q < gfirst + kept; ++q) B->segs[q].gcount = (int16_t)kept;
            // nearest other ranges of the group (the pileup's one-range weight shortcut)
            for (int32_t q = gfirst; q < gfirst + kept; ++q) {
                RcpSeg& a = B->segs[q];
                a.nb_lo = INT32_MIN;
                a.nb_hi = INT32_MAX;
                if (!multi) continue;
                for (int32_t t = gfirst; t < gfirst + kept; ++t) {
                    if (t == q || !B->segs[t].query_ok) continue;
                    const RcpSeg& b = B->segs[t];
                    if (b.hi < a.lo) a.nb_lo = std::max(a.nb_lo, b.hi);
                    else if (b.lo > a.hi) a.nb_hi = std::min(a.nb_hi, b.lo);
                    else a.nb_lo = INT32_MAX;  // intersecting ranges: always count
                }
            }
            g0 = g1;
        }
        B->row_len[r] = off;
    }
    B->row_seg[R] = (int32_t)B->segs.size();
    return RCP_OK;
}

template <class T>
size_t put(std::vector<char>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 255) & ~size_t(255);
    blob.resize(off + sizeof(T) * std::max<size_t>(v.size(), 1));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), sizeof(T) * v.size());
    return off;
}

// The plan's device tables as one arena: pieces are laid out (256-B aligned) and then copied
// straight from the host vectors through the pinned staging buffers (rcp_stage.h) -- no host
// blob to assemble (C4: 26 MB, ~15 ms of host copies and page faults into a fresh vector).
struct Arena {
    struct Piece {
        const void* p;
        size_t bytes, off;
    };
    std::vector<Piece> pieces;
    size_t total = 0;
    template <class T>
    size_t add(const std::vector<T>& v) {
        const size_t off = (total + 255) & ~size_t(255);
        if (!v.empty()) pieces.push_back({v.data(), sizeof(T) * v.size(), off});
        total = off + sizeof(T) * std::max<size_t>(v.size(), 1);
        return off;
    }
    hipError_t upload(void* dev, int device, hipStream_t s) const {
        for (const Piece& q : pieces) {
            const hipError_t e = rcp::stage_h2d(static_cast<char*>(dev) + q.off, q.p, q.bytes, device, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
};

}  // namespace

extern "C" int rcp_plan_create(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins,
                               rcp_plan** out) {
    RCP_TRY
    return rcp_plan_create_ex(rs, rows, bins, nullptr, out);
    RCP_CATCH
}

extern "C" int rcp_plan_create_ex(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins,
                                  const rcp_plan_opts* opts, rcp_plan** out) {
    RCP_TRY
    if (!rs || !rows || !out) return fail(RCP_EINVAL, "NULL argument");
    const rcp_plan_opts default_opts{RCP_KERNEL_AUTO, -1, 0, 0, 0, {0, 0}};
    if (!opts) opts = &default_opts;
    if (opts->pileup_kernel < RCP_KERNEL_AUTO || opts->pileup_kernel > RCP_KERNEL_BINS)
        return fail(RCP_EINVAL, "pileup_kernel = %d", opts->pileup_kernel);
    if (opts->concurrent < 0) return fail(RCP_EINVAL, "concurrent = %d", opts->concurrent);
    *out = nullptr;
    const rcp_bins_desc coverage_only{};  // bins == NULL: a calcCoverage-only plan
    const bool cov_only = bins == nullptr;
    if (cov_only) bins = &coverage_only;
    if (rows->n_rows < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (rows->n_rows > 0 && (!rows->seg_off || !rows->seg_chrom || !rows->seg_start || !rows->seg_end || !rows->seg_strand))
        return fail(RCP_EINVAL, "NULL row array");
    if (!cov_only && (bins->n_parts < 1 || bins->n_parts > RCP_MAX_PARTS))
        return fail(RCP_EINVAL, "n_parts = %d", bins->n_parts);
    if (bins->stat != RCP_STAT_MEAN && bins->stat != RCP_STAT_MEDIAN) return fail(RCP_EINVAL, "stat = %d", bins->stat);
    if (bins->interp < 0 || bins->interp > 3) return fail(RCP_EINVAL, "interp = %d", bins->interp);
    const bool rounding = bins->rng_kind == RCP_RNG_ROUNDING;
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);

    PlanTimer ptimer;
    if (!rows->ignore_strand) {  // findOverlaps with strand compatibility: the stranded layout
        const int rc0 = ensure_stranded(rs);
        if (rc0) return rc0;
    } else if (!rs->has_merged) {
        return fail(RCP_EINVAL, "this readset holds no strand-merged layout (a shard built for ignore.strand = FALSE)");
    }
    auto plan = std::make_unique<rcp_plan>();
    plan->rs = rs;
    Builder B;
    int rc = build_rows(rs, rows, &B);
    if (rc) return rc;
    const int R = rows->n_rows;
    PLAN_MARK("build_rows");
    plan->n_rows = R;
    plan->n_seg = (int64_t)B.segs.size();
    plan->row_len.assign(B.row_len.begin(), B.row_len.end());
    for (int r = 0; r < R; ++r) plan->max_row_len = std::max(plan->max_row_len, B.row_len[r]);

    RcpPlanDev& P = plan->dev;
    P.multi_rows = 0;
    for (int r = 0; r < R && !P.multi_rows; ++r) P.multi_rows = B.row_seg[r + 1] - B.row_seg[r] > 1;
    // persistent pileup grids: all workgroup slots alone, 7/8 beside other samples in flight
    // (rcp_plan_opts.concurrent; profiles/r04/r4p)
    P.grid_fill = opts->concurrent > 1 ? 7 : 8;
    P.n_parts = bins->n_parts;
    P.stat = bins->stat;
    P.scale = bins->scale;
    int64_t col = 0;
    int32_t chunk_cap = 1024, stage_cap = 1;
    bool lean_ok = true;  // so far: uniform power-of-two bins (no R-RNG layouts)
    int32_t max_interp_len = 0, max_interp_bins = 0;
    std::vector<int32_t> part_max_bin(RCP_MAX_PARTS, 1);
    std::map<std::pair<int, int>, int32_t> layout_cache;  // (n, dif) -> offset in lay_cnt
    std::map<std::pair<int, int>, int32_t> nb_cache;      // (n, L) -> offset in nb_pos
    for (int p = 0; p < bins->n_parts; ++p) {
        RcpPart& pt = P.part[p];
        const int32_t f1 = bins->flank[0], f2 = bins->flank[1];
        if (f1 < 0 || f2 < 0) return fail(RCP_EINVAL, "negative flank");
        switch (bins->where ? bins->where[p] : RCP_WHERE_WHOLE) {
            case RCP_WHERE_WHOLE: pt.lo_off = 0; pt.lo_end = 0; pt.hi_off = 0; pt.hi_end = 1; break;
            case RCP_WHERE_CENTER: pt.lo_off = f1; pt.lo_end = 0; pt.hi_off = -f2; pt.hi_end = 1; break;
            case RCP_WHERE_UPSTREAM: pt.lo_off = 0; pt.lo_end = 0; pt.hi_off = f1; pt.hi_end = 0; break;
            case RCP_WHERE_DOWNSTREAM: pt.lo_off = -f2; pt.lo_end = 1; pt.hi_off = 0; pt.hi_end = 1; break;
            default: return fail(RCP_EINVAL, "where[%d] = %d", p, bins->where[p]);
        }
        const int nb = bins->n_bins[p];
        if (nb < 0) return fail(RCP_EINVAL, "n_bins[%d] < 0", p);
        pt.per_base = nb == 0;
        pt.n_bins = pt.per_base ? (bins->per_base_width ? bins->per_base_width[p] : 0) : nb;
        if (pt.n_bins <= 0) return fail(RCP_EINVAL, "part %d has no columns", p);
        pt.col_off = (int32_t)col;
        col += pt.n_bins;
        pt.lay_base = (int32_t)B.lay_index.size();
        int32_t max_bin = 1;
        if (!pt.per_base) {
            B.lay_index.resize(B.lay_index.size() + pt.n_bins, -1);
            for (int r = 0; r < R; ++r) {
                int32_t head, L;
                rcp_part_slice(pt, B.row_len[r], &head, &L);
                if (B.row_static[r] || B.row_seg[r] == B.row_seg[r + 1]) continue;  // always NULL
                if (L < 0 || head < 0 || head + L > B.row_len[r])
                    return fail(RCP_EUNSUPPORTED, "row %d: part %d slice out of its %d-long coverage", r, p,
                                B.row_len[r]);
                if (L < pt.n_bins) {
                    int mode = bins->interp;
                    if (mode == RCP_INTERP_AUTO)
                        mode = ((double)(pt.n_bins - L) / pt.n_bins < 0.2) ? RCP_INTERP_NEIGHBORHOOD : RCP_INTERP_SPLINE;
                    int32_t pos_off = -1;
                    if (mode == RCP_INTERP_NEIGHBORHOOD) {
                        auto key = std::make_pair(pt.n_bins, L);
                        auto it = nb_cache.find(key);
                        if (it == nb_cache.end()) {
                            std::vector<int32_t> pos;
                            if (!rcp::neighborhood_positions(pt.n_bins, L, rounding, &pos))
                                return fail(RCP_ESEMANTIC,
                                            "splitVector neighborhood interpolation of %d values into %d bins: R raises an error",
                                            L, pt.n_bins);
                            pos_off = (int32_t)B.nb_pos.size();
                            B.nb_pos.insert(B.nb_pos.end(), pos.begin(), pos.end());
                            nb_cache[key] = pos_off;
                        } else {
                            pos_off = it->second;
                        }
                    } else if (mode == RCP_INTERP_SPLINE && L < 1) {
                        return fail(RCP_ESEMANTIC, "spline() of zero points: R raises an error");
                    } else if (mode == RCP_INTERP_LINEAR && L < 1) {
                        return fail(RCP_EUNSUPPORTED, "empty slice with the 'linear' interpolation");
                    }
                    B.interp_row.push_back(r);
                    B.interp_part.push_back(p);
                    B.interp_mode.push_back(mode);
                    B.interp_pos.push_back(pos_off);
                    max_interp_len = std::max(max_interp_len, L);
                    max_interp_bins = std::max(max_interp_bins, pt.n_bins);
                    continue;
                }
                const int32_t bs = L / pt.n_bins;
                const int32_t dif = L - bs * pt.n_bins;
                if (dif || (bs & (bs - 1))) lean_ok = false;
                // median bins wider than a wave chunk go to the slow-row kernel (mode 4) and do
                // not size the chunks of the others
                if (bins->stat != RCP_STAT_MEDIAN || bs + (dif ? 1 : 0) < kWaveMax)
                    max_bin = std::max(max_bin, bs + (dif ? 1 : 0));
                if (dif) {
                    int32_t& slot = B.lay_index[pt.lay_base + dif];
                    if (slot < 0) {
                        auto key = std::make_pair(pt.n_bins, dif);
                        auto it = layout_cache.find(key);
                        if (it == layout_cache.end()) {
                            const std::vector<int32_t> cnt = rcp::bin_layout_counts(pt.n_bins, dif, rounding);
                            const int32_t o = (int32_t)B.lay_cnt.size();
                            B.lay_cnt.insert(B.lay_cnt.end(), cnt.begin(), cnt.end());
                            B.lay_regions.emplace_back(o, pt.n_bins);
                            layout_cache[key] = o;
                            slot = o;
                        } else {
                            slot = it->second;
                        }
                    }
                }
            }
        }
        part_max_bin[p] = max_bin;
    }
    if (max_interp_len > kChunkMax)
        return fail(RCP_EUNSUPPORTED, "interpolated slice of %d positions exceeds %d", max_interp_len, kChunkMax);

    // ---- geometry.  A workgroup handles <= kStageMaxBins bins of a part for 32 rows; a wave
    // piles a row's positions for those bins in sub-chunks of at most `chunk_cap` positions
    // (bins straddling sub-chunks accumulate).  Pick the largest wave chunk (<= kWaveMax) whose
    // LDS (4 wave arrays + [bin][row] stage + row metadata) keeps two workgroups per CU.
    {
        const bool median = bins->stat == RCP_STAT_MEDIAN;
        int32_t need = 64;
        for (int p = 0; p < P.n_parts; ++p) {
            RcpPart& pt = P.part[p];
            // equal chunks of at most kStageMaxBins bins
            int32_t nch = (pt.n_bins + kStageMaxBins - 1) / kStageMaxBins;
            int32_t cb = (pt.n_bins + nch - 1) / nch;
            // wide binned chunks would be piled in several wave sub-chunks, each streaming the
            // chunk's reads again: split them into more (up to 8) column chunks instead -- more
            // workgroups for small row counts, and per-chunk read ranges from locate.  The general
            // kernel's cap stays at the 8 chunks its A/B measured (lean plans split further, to
            // RCP_MAX_CRANGE_CHUNKS, below)
            const int32_t pos_max = 1023;
            if (!median && !pt.per_base && part_max_bin[p] > 0 && (int64_t)cb * part_max_bin[p] > pos_max) {
                const int32_t cb2 = std::max<int32_t>(1, pos_max / part_max_bin[p]);
                const int32_t nch2 = (pt.n_bins + cb2 - 1) / cb2;
                if (nch2 <= kGeneralMaxChunks) {
                    nch = nch2;
                    cb = (pt.n_bins + nch - 1) / nch;
                }
            }
            // opts->min_col_chunks (one-part plans): at least that many column chunks
            if (!median && P.n_parts == 1 && opts->min_col_chunks > nch) {
                nch = std::min<int32_t>(std::min(opts->min_col_chunks, RCP_MAX_CRANGE_CHUNKS), pt.n_bins);
                cb = (pt.n_bins + nch - 1) / nch;
            }
            if (median) cb = std::min<int32_t>(cb, std::max<int32_t>(1, kWaveMax / part_max_bin[p]));
            pt.chunk_bins = cb;
            pt.n_chunks = (pt.n_bins + cb - 1) / cb;
            stage_cap = std::max(stage_cap, cb);
            need = std::max<int64_t>(need, std::min<int64_t>((int64_t)cb * part_max_bin[p], kWaveMax));
        }
        if (cov_only) need = std::max(need, std::min(plan->max_row_len, kWaveMax));
        int32_t min_cap = 64;
        if (median)
            for (int p = 0; p < P.n_parts; ++p) min_cap = std::max(min_cap, P.part[p].chunk_bins * part_max_bin[p]);
        const int32_t cands[] = {need, 2047, 1023, 511};  // 64 * 2^k - 1: the +1 sentinel fits
        chunk_cap = -1;
        for (int32_t ch : cands) {
            if (ch > need || ch < min_cap) continue;
            RcpPlanDev t{};
            int32_t cap_unused = 0;
            wave_geometry(ch, &t.wave_words, &cap_unused);
            t.stage_cap = cov_only ? 0 : stage_cap;
            chunk_cap = ch;
            if (rcp_pileup_lds_bytes(&t, cov_only ? 1 : 0) <= kLdsBudget) break;
        }
        if (chunk_cap < 0) chunk_cap = need;
    }
    P.n_cols = col;
    plan->n_cols = col;
    if (opts->out_ld == RCP_OUT_LD_PADDED) P.out_ld = ((int64_t)R + 15) & ~int64_t(15);
    else if (opts->out_ld == 0) P.out_ld = R;
    else if (opts->out_ld >= R) P.out_ld = opts->out_ld;
    else return fail(RCP_EINVAL, "out_ld = %lld < n_rows = %d", (long long)opts->out_ld, R);
    plan->out_ld = P.out_ld;
    wave_geometry(chunk_cap, &P.wave_words, &P.chunk_cap);
    P.stage_cap = stage_cap;
    P.interp_cap = std::max(max_interp_len, 1);
    if (bins->stat == RCP_STAT_MEDIAN) {
        // rows whose median bins exceed the wave chunk: block-level windows (mode 4)
        for (int p = 0; p < P.n_parts; ++p) {
            const RcpPart& pt = P.part[p];
            if (pt.per_base) continue;
            for (int r = 0; r < R; ++r) {
                if (B.row_static[r] || B.row_seg[r] == B.row_seg[r + 1]) continue;
                int32_t head, L;
                rcp_part_slice(pt, B.row_len[r], &head, &L);
                if (L < pt.n_bins) continue;
                const int32_t bs = L / pt.n_bins, dif = L - bs * pt.n_bins;
                const int32_t w = bs + (dif ? 1 : 0);
                if (w <= P.chunk_cap) continue;
                if (w > kChunkMax)
                    return fail(RCP_EUNSUPPORTED, "row %d: a median bin of %d positions exceeds %d", r, w, kChunkMax);
                B.interp_row.push_back(r);
                B.interp_part.push_back(p);
                B.interp_mode.push_back(4);
                B.interp_pos.push_back(dif ? B.lay_index[pt.lay_base + dif] : -1);
                P.interp_cap = std::max(P.interp_cap, w);
            }
        }
    }
    P.n_chunks_total = 0;
    for (int p = 0; p < P.n_parts; ++p) P.n_chunks_total += P.part[p].n_chunks;

    // ---- lean pileup kernel: every row one plain range (no exon list, no zero-width query),
    // mean of uniform power-of-two bins, each chunk inside one wave's fused pass (<= 1023
    // positions) and the stage inside the store waves' registers
    // With opts->pileup_kernel == RCP_KERNEL_LEAN_ANY, other plans take its general-bins mode
    // (lean == 2): any uniform width, R-RNG layouts and multi-range rows, as long as every chunk
    // is one wave's pass (no sub-chunks) and holds <= rcp_lean_gen_max_bins() bins.  Measured
    // slower than the general kernel on C2 (0.082 vs 0.063 ms) and C3 (0.96 vs 0.88 ms), so
    // AUTO does not choose it.  RCP_KERNEL_GENERAL keeps every plan on the general kernel.
    bool lean_base = false;  // a lean plan whose every part is per base
    {
        const int kind = opts->pileup_kernel;
        bool base = !cov_only && bins->stat == RCP_STAT_MEAN && P.chunk_cap <= 1023 && kind != RCP_KERNEL_GENERAL;
        for (int p = 0; base && p < P.n_parts; ++p) {
            const RcpPart& pt = P.part[p];
            const int64_t w = pt.per_base ? 1 : part_max_bin[p];
            if ((int64_t)pt.chunk_bins * w > P.chunk_cap) base = false;
        }
        bool lean = base && lean_ok && stage_cap <= rcp_lean_max_bins();
        if (lean && kind == RCP_KERNEL_AUTO && R < kLeanMinRowsBinned) {
            bool binned = true;
            for (int p = 0; p < P.n_parts; ++p) binned = binned && !P.part[p].per_base;
            if (binned) lean = false;
        }
        for (int r = 0; lean && r < R; ++r) {
            const int32_t j0 = B.row_seg[r], j1 = B.row_seg[r + 1];
            if (j1 - j0 > 1) lean = false;
            else if (j1 == j0 + 1 && (B.segs[j0].multi || !B.segs[j0].query_ok)) lean = false;
        }
        const bool gen = !lean && base && kind == RCP_KERNEL_LEAN_ANY &&
                         stage_cap <= rcp_lean_gen_max_bins();
        P.lean = lean ? 1 : (gen ? 2 : 0);
        {
            bool per_base = true;
            for (int p = 0; p < P.n_parts; ++p) per_base = per_base && P.part[p].per_base;
            lean_base = P.lean && per_base;
            P.lean_rounds = lean_base ? 2 : 0;
            // (RCP_LEAN_ROUNDS=2: diagnostics A/B of two-round items for binned lean plans)
            if (P.lean && !per_base && std::getenv("RCP_LEAN_ROUNDS") && std::atoi(std::getenv("RCP_LEAN_ROUNDS")) == 2)
                P.lean_rounds = 2;
        }
        // row-wave kernel (lean == 3): mean bins of any layout, every bin inside one window;
        // AUTO takes it for plans with multi-range rows (coverageRnaRef, genebody + flanks)
        bool rows_ok = !cov_only && bins->stat == RCP_STAT_MEAN && kind != RCP_KERNEL_GENERAL && !lean;
        for (int p = 0; rows_ok && p < P.n_parts; ++p)
            if (!P.part[p].per_base && part_max_bin[p] > rcp_rows_window_cap()) rows_ok = false;
        bool multi_rows = false;
        for (int r = 0; !multi_rows && r < R; ++r) multi_rows = B.row_seg[r + 1] - B.row_seg[r] > 1;
        if (rows_ok && (kind == RCP_KERNEL_ROWS || (kind == RCP_KERNEL_AUTO && multi_rows))) {
            P.lean = 3;
            // each wave searches its rows' (segment, stream) ranges itself (no locate launch, no
            // 64-B record round trip; a skewed row stays with the wave that claimed it) unless
            // the caller asked for the heavy path
            P.fold = opts->heavy_threshold <= 0 ? 1 : 0;
        }
    }
    // ---- bin-difference kernel (lean == 4): mean plans of one binned part whose rows are
    // single ranges, every row's slice a whole number of bins of >= rcp_bins_min_width()
    // positions (no splitVector layout, no interpolation), <= rcp_bins_max_bins() bins.  A row
    // is one wave's pass over its bins (no column chunks).  AUTO takes it for such plans:
    // C2 (200 bins of 20 bp) ... ; RCP_KERNEL_BINS forces it where the shape allows
    {
        const int kind = opts->pileup_kernel;
        bool bd = !cov_only && bins->stat == RCP_STAT_MEAN && P.n_parts == 1 && !P.part[0].per_base &&
                  P.part[0].n_bins > 0 && P.part[0].n_bins <= rcp_bins_max_bins() &&
                  (kind == RCP_KERNEL_AUTO || kind == RCP_KERNEL_BINS);
        const RcpPart& pt0 = P.part[0];
        for (int r = 0; bd && r < R; ++r) {
            const int32_t j0 = B.row_seg[r], j1 = B.row_seg[r + 1];
            if (B.row_static[r] || j1 == j0) continue;  // NULL rows: zeros
            if (j1 - j0 > 1 || B.segs[j0].multi || !B.segs[j0].query_ok) {
                bd = false;
                break;
            }
            int32_t head, L;
            rcp_part_slice(pt0, B.row_len[r], &head, &L);
            if (L < pt0.n_bins || L % pt0.n_bins != 0 || L / pt0.n_bins < rcp_bins_min_width()) bd = false;
        }
        if (bd && B.interp_row.empty()) {
            P.lean = 4;
            P.part[0].chunk_bins = P.part[0].n_bins;
            P.part[0].n_chunks = 1;
            P.n_chunks_total = 1;
            P.stage_cap = P.part[0].n_bins;
            // the kernel searches its rows' read ranges itself (the locate and heavy launches
            // were as long as the pileup on C2) unless the caller asked for the heavy path
            P.fold = opts->heavy_threshold <= 0 ? 1 : 0;
        }
    }
    // ---- general-kernel plans of small tables of single ranges in the merged layout (one GPU's
    // shard of a peak table: C4 1/8 spent locate 25 + heavy 8 us ahead of a 93-us pileup): the
    // pileup kernel searches each row's and chunk's read ranges itself (fold_row) and piles a
    // skewed row with the whole workgroup instead of heavy slices -- unless the caller asked for
    // the heavy path.  Every chunk must be one wave pass (no sub-chunks: those read locate's
    // segment ranges) and no row interpolated (rcp_interp_kernel reads them too)
    if (P.lean == 0 && !cov_only && rows->ignore_strand && opts->heavy_threshold <= 0 && B.interp_row.empty() &&
        R > 0 && R <= kFoldMaxRows) {
        bool f = true;
        for (int p = 0; f && p < P.n_parts; ++p) {
            const RcpPart& pt = P.part[p];
            const int64_t w = pt.per_base ? 1 : part_max_bin[p];
            if ((int64_t)pt.chunk_bins * w > P.chunk_cap) f = false;
        }
        for (int r = 0; f && r < R; ++r) {
            const int32_t j0 = B.row_seg[r], j1 = B.row_seg[r + 1];
            if (B.row_static[r] || j1 == j0) continue;  // NULL rows
            if (j1 - j0 > 1 || B.segs[j0].multi || !B.segs[j0].query_ok) f = false;
        }
        P.fold = f ? 1 : 0;
    }
    // ---- per-base lean plans of small tables in the merged layout (one GPU's shard of a per-base
    // table: C5 1/8 spent locate 45 us ahead of a 143-us pileup): the store wave that claims an
    // item searches its rows' read ranges while the pile waves work on the previous item -- no
    // locate launch.  (Binned lean plans keep the locate: their skewed rows need the heavy slices.)
    // Plans built for several samples in flight (rcp_plan_opts.concurrent) of a larger table keep
    // the locate launch: it runs beside another sample's pileup there, while the claim's searches
    // lengthen this kernel (full C5 at D = 2: 0.459-0.463 vs 0.472-0.480 ms a step).
    if (P.lean == 1 && lean_base && rows->ignore_strand && opts->heavy_threshold <= 0 &&
        B.interp_row.empty() && R > 0 && R <= kFoldMaxRows && (opts->concurrent <= 1 || R <= kFoldConcurrentMaxRows) &&
        !std::getenv("RCP_NO_LEAN_FOLD")) {
        bool f = true;
        for (int r = 0; f && r < R; ++r) {
            const int32_t j0 = B.row_seg[r], j1 = B.row_seg[r + 1];
            if (B.row_static[r] || j1 == j0) continue;
            if (j1 - j0 > 1 || B.segs[j0].multi || !B.segs[j0].query_ok) f = false;
        }
        P.fold = f ? 1 : 0;
    }
    // (RCP_COOP_MIN: diagnostics A/B of the cooperative rows' threshold)
    P.coop_min = std::getenv("RCP_COOP_MIN") ? std::max(0, std::atoi(std::getenv("RCP_COOP_MIN"))) : kCoopMin;
    // ---- lean plans with few row tiles (one GPU's shard of a region table): the persistent
    // grid (two workgroups per CU) takes (row tile, column chunk) items; with few items per
    // workgroup the last ones leave most workgroups idle, so cut the parts into more column
    // chunks (each streams only its reads: crange) until there are >= kLeanItemsPerWg per
    // workgroup, or opts->min_col_chunks asks for more
    if (P.lean == 1 && R > 0) {
        int cus = 256;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, rs->device) != hipSuccess || cus <= 0)
            cus = 256;
        const int64_t grid = (2 * (int64_t)cus + 7) / 8 * 8;
        const int64_t trows = P.lean_rounds == 2 ? 32 : rcp_tile_rows();
        const int64_t tiles = ((int64_t)R + trows - 1) / trows;
        auto can_split = [&]() {
            if (P.n_chunks_total * 2 > RCP_MAX_CRANGE_CHUNKS) return false;
            for (int p = 0; p < P.n_parts; ++p)
                if (P.part[p].chunk_bins < 2 * kLeanMinChunkBins) return false;
            return true;
        };
        auto split = [&]() {
            P.n_chunks_total = 0;
            for (int p = 0; p < P.n_parts; ++p) {
                RcpPart& pt = P.part[p];
                const int32_t nch = 2 * pt.n_chunks;
                pt.chunk_bins = (pt.n_bins + nch - 1) / nch;
                pt.n_chunks = (pt.n_bins + pt.chunk_bins - 1) / pt.chunk_bins;
                P.n_chunks_total += pt.n_chunks;
            }
        };
        const int64_t want = (lean_base ? kLeanItemsPerWgBase : kLeanItemsPerWg) * grid;
        while (can_split() && (tiles * P.n_chunks_total < want || P.n_chunks_total < opts->min_col_chunks))
            split();
        P.stage_cap = 1;
        for (int p = 0; p < P.n_parts; ++p) P.stage_cap = std::max(P.stage_cap, P.part[p].chunk_bins);
    }

    PLAN_MARK("parts+geometry");
    // ---- skewed rows: heavy slots sized for the eligible (short enough) rows
    const int32_t heavy_thr = opts->heavy_threshold < 0 ? kHeavyThreshold : opts->heavy_threshold;
    int32_t eligible_len = 0;
    for (int r = 0; r < R; ++r)
        if (B.row_len[r] <= kHeavyMaxLen) eligible_len = std::max(eligible_len, B.row_len[r]);
    P.heavy_threshold = heavy_thr;
    P.heavy_max_len = eligible_len;
    P.heavy_stride = ((eligible_len + 1) + 63) & ~63;
    P.heavy_slice = kHeavySlice;
    P.heavy_cap = (int32_t)std::min<int64_t>(std::max(R, 1), std::min<int64_t>(4096, (256ll << 20) / (4ll * P.heavy_stride)));
    if (heavy_thr <= 0 || R == 0 || P.fold) P.heavy_threshold = 0;

    // ---- upload tables (one arena)
    Arena blob;
    const size_t o_row_chrom = blob.add(B.row_chrom);
    const size_t o_row_seg = blob.add(B.row_seg);
    const size_t o_row_len = blob.add(B.row_len);
    const size_t o_row_static = blob.add(B.row_static);
    const size_t o_segs = blob.add(B.segs);
    const size_t o_lay_index = blob.add(B.lay_index);
    const size_t o_lay_cnt = blob.add(B.lay_cnt);
    // the same layouts as bit masks (word lay + j: bins 32 j .. 32 j + 31 enlarged), indexed
    // like lay_cnt: one load per 32 bins where the row-wave flush needs the bin widths
    std::vector<uint32_t> lay_bit(B.lay_cnt.size(), 0u);
    for (const auto& rg : B.lay_regions)
        for (int32_t k = 0; k < rg.second; ++k)
            if (B.lay_cnt[rg.first + k + 1] != B.lay_cnt[rg.first + k]) lay_bit[rg.first + (k >> 5)] |= 1u << (k & 31);
    const size_t o_lay_bit = blob.add(lay_bit);
    const size_t o_irow = blob.add(B.interp_row);
    const size_t o_ipart = blob.add(B.interp_part);
    const size_t o_imode = blob.add(B.interp_mode);
    const size_t o_ipos = blob.add(B.interp_pos);
    // row-wave plans interpolate the rows they pile (rcp_pileup_rows_kernel): entry of (row, part)
    std::vector<int32_t> interp_of;
    if (P.lean == 3 && !B.interp_row.empty()) {
        interp_of.assign((size_t)R * P.n_parts, -1);
        for (size_t e = 0; e < B.interp_row.size(); ++e)
            interp_of[(size_t)B.interp_row[e] * P.n_parts + B.interp_part[e]] = (int32_t)e;
    }
    const size_t o_iof = blob.add(interp_of);
    // ... and claim the 16-row tiles holding such rows first, most first: the spline's serial
    // chains then run beside the other waves' pileup, not in the grid's tail
    std::vector<int32_t> tile_perm;
    if (!interp_of.empty()) {
        const int32_t n_tiles = (R + 15) / 16;
        std::vector<int32_t> cnt(n_tiles, 0);
        for (int32_t r : B.interp_row) ++cnt[r / 16];
        tile_perm.resize(n_tiles);
        for (int32_t t = 0; t < n_tiles; ++t) tile_perm[t] = t;
        std::stable_sort(tile_perm.begin(), tile_perm.end(), [&](int32_t a, int32_t b) { return cnt[a] > cnt[b]; });
    }
    const size_t o_tperm = blob.add(tile_perm);
    const size_t o_nb = blob.add(B.nb_pos);
    // locate's per-row input (RcpRowInfo)
    std::vector<RcpRowInfo> row_info((size_t)std::max(R, 1));
    {
        const ReadLayout& RL0 = rows->ignore_strand ? rs->merged : rs->stranded;
        for (int r = 0; r < R; ++r) {
            RcpRowInfo& ri = row_info[r];
            std::memset(&ri, 0, sizeof(ri));
            ri.j0 = B.row_seg[r];
            ri.j1 = B.row_seg[r + 1];
            ri.chrom = B.row_chrom[r];
            ri.row_len = B.row_len[r];
            ri.stat = B.row_static[r];
            const bool cok = ri.chrom >= 0 && ri.chrom < rs->n_chrom;
            ri.seqlen = cok ? rs->seqlen[ri.chrom] : -1;
            if (cok) {
                ri.d0 = RL0.h_dir_off[(size_t)ri.chrom * 3];
                ri.nb = (int32_t)(RL0.h_dir_off[(size_t)ri.chrom * 3 + 1] - ri.d0) - 1;
            }
            if (ri.j1 > ri.j0) ri.seg0 = B.segs[ri.j0];
        }
    }
    const size_t o_rinfo = blob.add(row_info);
    // fmm pivots (see RcpPlanDev::spl_tb): the elimination of R's fmm_spline with d[i] = 1
    std::vector<double> spl_tb(2 * ((size_t)std::max(max_interp_len, 1) + 1), 0.0);
    {
        double bp = -1.0;
        spl_tb[1] = bp;
        for (size_t i = 1; 2 * i + 1 < spl_tb.size(); ++i) {
            const double t = 1.0 / bp;
            bp = 4.0 - t;
            spl_tb[2 * i] = t;
            spl_tb[2 * i + 1] = bp;
        }
    }
    const size_t o_spl = blob.add(spl_tb);
    PLAN_MARK("tables (host)");
    HIP_TRY(plan->tables.alloc(blob.total, nullptr));
    HIP_TRY(blob.upload(plan->tables.p, rs->device, nullptr));
    PLAN_MARK("tables upload");
    char* base = plan->tables.as<char>();
    // ---- work arena: locate outputs, heavy-row state, status words
    const int64_t S = std::max<int64_t>(plan->n_seg, 1);
    const int64_t Rw = std::max(R, 1);
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t w_lo = 0;
    const size_t w_hi = al(w_lo + 12 * S);
    const size_t w_valid = al(w_hi + 12 * S);
    const size_t w_ncand = al(w_valid + Rw);
    const size_t w_hrows = al(w_ncand + 4 * Rw);
    const size_t w_hoff = al(w_hrows + 4 * (size_t)P.heavy_cap);
    const size_t w_gdiff = al(w_hoff + 4 * ((size_t)P.heavy_cap + 1));
    const size_t w_rec = al(w_gdiff + (P.heavy_threshold > 0 ? 4 * (size_t)P.heavy_cap * P.heavy_stride : 0));
    const bool keep_crange = P.n_chunks_total > 1 && P.n_chunks_total <= RCP_MAX_CRANGE_CHUNKS;
    const size_t w_crange = al(w_rec + sizeof(RcpRowRec) * Rw);
    // heaviest-first lean items (rcp_device.h lpt): per-base lean plans of few 32-row items,
    // i.e. one GPU's shard of a per-base table (C5 1/8: TSS windows' middle column chunks hold
    // several times the outer chunks' reads; in per-XCD order a workgroup that drew two heavy
    // items sets the pass)
    const int64_t lpt_items = ((int64_t)R + 31) / 32 * P.n_chunks_total;
    int lpt_cus = 256;
    if (hipDeviceGetAttribute(&lpt_cus, hipDeviceAttributeMultiprocessorCount, rs->device) != hipSuccess || lpt_cus <= 0)
        lpt_cus = 256;
    // (a full per-base table, e.g. C5's 6256 items, keeps the per-XCD order and its L2 locality)
    P.lpt = P.lean == 1 && lean_base && keep_crange && R > 0 && !P.fold &&
            lpt_items <= (int64_t)kLeanItemsPerWgBase * 2 * lpt_cus;
    P.lpt_cap = P.lpt ? (int32_t)lpt_items : 0;
    const size_t w_order = al(w_crange + (keep_crange ? sizeof(uint2) * 3 * (size_t)P.n_chunks_total * Rw : 0));
    const size_t w_status = al(w_order + 4 * (size_t)RCP_LPT_CLASSES * (size_t)P.lpt_cap);
    static_assert(2 * RCP_STATUS_WORDS * 4 <= 256, "two status sets");
    HIP_TRY(plan->work.alloc(w_status + 256, nullptr));
    PLAN_MARK("work alloc");
    char* wb = plan->work.as<char>();
    P.ncand = reinterpret_cast<uint32_t*>(wb + w_ncand);
    P.heavy_rows = reinterpret_cast<int32_t*>(wb + w_hrows);
    P.heavy_nslice = reinterpret_cast<uint32_t*>(wb + w_hoff);
    P.heavy_gdiff = reinterpret_cast<int32_t*>(wb + w_gdiff);
    P.rec = reinterpret_cast<RcpRowRec*>(wb + w_rec);
    P.crange = keep_crange ? reinterpret_cast<uint2*>(wb + w_crange) : nullptr;
    P.item_order = P.lpt ? reinterpret_cast<int32_t*>(wb + w_order) : nullptr;
    // the locate kernel's chunk windows for the rows of the first row's length (all rows of
    // C2 / C4 / C5), when no part of that length has an R-RNG layout: the same arithmetic as
    // the kernel's chunk_window, once per plan instead of once per (row, chunk)
    P.cw_len = -1;
    if (keep_crange && R > 0) {
        const int32_t nr = B.row_len[0];
        bool ok = true;
        int c = 0;
        for (int p = 0; ok && p < P.n_parts; ++p) {
            const RcpPart& pt = P.part[p];
            for (int cp = 0; cp < pt.n_chunks; ++cp, ++c) {
                int32_t head, L;
                rcp_part_slice(pt, nr, &head, &L);
                const int32_t n = pt.n_bins, k0 = cp * pt.chunk_bins;
                P.cw[2 * c] = 0;
                P.cw[2 * c + 1] = -1;
                if (k0 >= n || (pt.per_base ? L != n : L < n)) continue;
                const int32_t bs = pt.per_base ? 1 : L / n;
                if (!pt.per_base && L - bs * n != 0) {
                    ok = false;  // an R-RNG layout: the kernel computes these rows itself
                    break;
                }
                if (P.stat == 1 && bs > P.chunk_cap) continue;
                const int32_t kend = std::min(k0 + pt.chunk_bins, n);
                P.cw[2 * c] = head + bs * k0;
                P.cw[2 * c + 1] = bs * (kend - k0);
            }
        }
        if (ok) P.cw_len = nr;
    }
    const int32_t n_interp = (int32_t)B.interp_row.size();
    // x (L+1) | b, c, d (3 (L+1)) for the spline, or the neighborhood fill's n pre-fill values
    P.interp_stride = (max_interp_len + 1) + std::max(max_interp_bins, 3 * (max_interp_len + 1)) + 8;
    if (n_interp) HIP_TRY(plan->scratch.alloc(8 * (size_t)n_interp * P.interp_stride, nullptr));

    const ReadLayout& RL = rows->ignore_strand ? rs->merged : rs->stranded;
    P.se = RL.se.as<int2>();
    // uniform-width reads: the general kernel and per-base lean plans stream the starts alone;
    // binned lean plans keep the (start, end) pairs -- C4's latency-bound pile measured 4 % slower
    // with starts (pileup 0.578 vs 0.555 ms, same box), C5's dense per-base rows 6 % faster
    // (0.58 vs 0.62), the 1/8 C4 shard's general kernel 4 % (profiles/r03/pipeline/general_starts_ab.log,
    // lean_starts_c4_ab.log)
    const bool use_st = RL.st.p && (P.lean != 1 || lean_base);
    P.st = use_st ? RL.st.as<int32_t>() : nullptr;
    P.st_w = RL.st_w;
    P.pmax = RL.pmax.as<int32_t>();
    P.stream_off = RL.stream_off.as<int64_t>();
    P.seqlen = rs->d_seqlen.as<int64_t>();
    P.dir_l = RL.dir_l.as<int32_t>();
    P.dir_u = RL.dir_l.as<int32_t>() + 1;  // interleaved with dir_l (stride 2)
    P.dir_off = RL.dir_off.as<int64_t>();
    P.dir_k = RL.dir_k.as<int32_t>();
    P.dir_shift = RL.dir_shift;
    P.merged = rows->ignore_strand ? 1 : 0;
    P.n_chrom = rs->n_chrom;
    P.n_rows = R;
    P.row_chrom = reinterpret_cast<const int32_t*>(base + o_row_chrom);
    P.row_seg = reinterpret_cast<const int32_t*>(base + o_row_seg);
    P.row_len = reinterpret_cast<const int32_t*>(base + o_row_len);
    P.row_static = reinterpret_cast<const uint8_t*>(base + o_row_static);
    P.segs = reinterpret_cast<const RcpSeg*>(base + o_segs);
    P.row_info = reinterpret_cast<const RcpRowInfo*>(base + o_rinfo);
    P.seg_lo = reinterpret_cast<uint32_t*>(wb + w_lo);
    P.seg_hi = reinterpret_cast<uint32_t*>(wb + w_hi);
    P.valid = reinterpret_cast<uint8_t*>(wb + w_valid);
    plan->status_sets = reinterpret_cast<uint32_t*>(wb + w_status);
    P.status = plan->status_sets;  // set by begin_exec per execution
    P.status_prev = plan->status_sets + RCP_STATUS_WORDS;
    P.lay_index = reinterpret_cast<const int32_t*>(base + o_lay_index);
    P.lay_cnt = reinterpret_cast<const int32_t*>(base + o_lay_cnt);
    P.lay_bit = reinterpret_cast<const uint32_t*>(base + o_lay_bit);
    P.n_interp = n_interp;
    P.interp_row = reinterpret_cast<const int32_t*>(base + o_irow);
    P.interp_part = reinterpret_cast<const int32_t*>(base + o_ipart);
    P.interp_mode = reinterpret_cast<const int32_t*>(base + o_imode);
    P.interp_pos = reinterpret_cast<const int32_t*>(base + o_ipos);
    P.interp_of = interp_of.empty() ? nullptr : reinterpret_cast<const int32_t*>(base + o_iof);
    P.tile_perm = tile_perm.empty() ? nullptr : reinterpret_cast<const int32_t*>(base + o_tperm);
    P.nb_pos = reinterpret_cast<const int32_t*>(base + o_nb);
    P.spl_tb = reinterpret_cast<const double*>(base + o_spl);
    P.interp_scratch = plan->scratch.as<double>();
    P.csr_off = nullptr;
    P.csr_out = nullptr;
    P.csr_rs = nullptr;
    P.csr_sub = nullptr;
    P.csr_sub_off = nullptr;
    // row-wave plans whose tile stage does not fit LDS stage their bin numerators row-major
    // (uint32 numerators, divided at the flush)
    P.rm32 = nullptr;
    P.rinfo = nullptr;
    if (P.lean == 3 && R > 0 && P.n_cols > 0) {
        HIP_TRY(plan->rm.alloc(4 * (size_t)R * (size_t)P.n_cols + 8 * (size_t)R * RCP_MAX_PARTS, nullptr));
        P.rinfo = plan->rm.as<int2>();
        P.rm32 = reinterpret_cast<uint32_t*>(P.rinfo + (size_t)R * RCP_MAX_PARTS);
    }
    plan->lds = P.lean == 4 ? rcp_pileup_bins_lds_bytes(&P)
                : P.lean == 3 ? rcp_pileup_rows_lds_bytes(&P)
                              : (P.lean ? rcp_pileup_lean_lds_bytes(&P) : rcp_pileup_lds_bytes(&P, cov_only ? 1 : 0));
    // the row-wave kernel's persistent grid holds one workgroup per CU for the whole pass: the
    // interpolation rows (a side stream, forked after locate) fit beside it only in the LDS it
    // leaves -- their spline arrays then go to global scratch (C3: 148 KB + 4 KB, vs 20 KB that
    // waited for the pileup to end)
    P.interp_lds_budget = P.lean == 3 ? (int32_t)std::max<int64_t>(0, 160 * 1024 - (int64_t)plan->lds) : 0;
    // general kernel: 2 rounds (32 rows) per workgroup (C3: 0.88 ms vs 0.91 with 4 rounds, 0.89
    // with 1), 1 when the row table is small, so that the grid still holds two workgroups per
    // CU (C2: 10k rows -> 625 workgroups instead of 157; pileup 0.076 -> 0.063 ms)
    {
        int tile = 16, rmax = 4;
        rcp_tile_geometry(&tile, &rmax);
        int cus = 256;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, rs->device) != hipSuccess || cus <= 0)
            cus = 256;
        P.n_cus = cus;
        P.rounds = std::min(rmax, 2);
        while (P.rounds > 1 &&
               (int64_t)((R + tile * P.rounds - 1) / (tile * P.rounds)) * P.n_chunks_total < 2 * (int64_t)cus)
            P.rounds /= 2;
        // (RCP_GEN_ROUNDS: diagnostics A/B of the rounds per workgroup, 1 / 2 / 4)
        if (const char* e = std::getenv("RCP_GEN_ROUNDS")) {
            const int v = std::atoi(e);
            if (v == 1 || v == 2 || v == 4) P.rounds = std::min(v, rmax);
        }
        plan->tile_rows = P.lean == 4 ? tile : (P.lean ? (P.lean_rounds == 2 ? 2 * tile : rcp_tile_rows()) : tile * P.rounds);
    }
    plan->grid = (int64_t)((R + plan->tile_rows - 1) / plan->tile_rows) * P.n_chunks_total;
    if (P.lean == 4) plan->grid = (plan->grid + 7) / 8 * 8;
    if (plan->lds > 160 * 1024) return fail(RCP_EUNSUPPORTED, "plan needs %zu B of LDS", plan->lds);
    PLAN_MARK("rest");
    // cleared before the plan is returned: its executions run on the caller's (non-blocking)
    // streams, which do not wait for the null stream
    HIP_TRY(hipMemsetAsync(plan->work.p, 0, plan->work.bytes, nullptr));
    HIP_TRY(hipStreamSynchronize(nullptr));
    PLAN_MARK("memset");
    *out = plan.release();
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_plan_destroy(rcp_plan* plan) {
    RCP_TRY
    if (!plan) return RCP_OK;
    DeviceGuard g(plan->rs->device);
    delete plan;
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_plan_info_get(const rcp_plan* plan, rcp_plan_info* info) {
    RCP_TRY
    if (!plan || !info) return fail(RCP_EINVAL, "NULL argument");
    info->n_cols = plan->n_cols;
    info->n_segments = plan->n_seg;
    info->n_interp_rows = plan->dev.n_interp;
    info->lds_bytes = (int64_t)plan->lds;
    info->grid = plan->grid;
    info->tile_rows = plan->tile_rows;
    info->chunk_positions = plan->dev.chunk_cap;
    info->pileup_kernel = plan->dev.lean;
    info->read_bytes = plan->dev.st ? 4 : 8;
    info->out_ld = plan->out_ld;
    info->fold = plan->dev.fold;
    info->reserved = 0;
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_plan_row_lengths(const rcp_plan* plan, int64_t* out_len) {
    RCP_TRY
    if (!plan || !out_len) return fail(RCP_EINVAL, "NULL argument");
    std::memcpy(out_len, plan->row_len.data(), 8 * plan->row_len.size());
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_plan_validity(rcp_plan* plan, uint8_t* d_valid, void* hip_stream) {
    RCP_TRY
    if (!plan) return fail(RCP_EINVAL, "NULL plan");
    DeviceGuard g(plan->rs->device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    begin_exec(plan);
    RcpPlanDev Q = plan->dev;
    Q.valid_out = d_valid;
    HIP_TRY(rcp_launch_locate(&Q, s));
    Q.heavy_threshold = 0;  // no slices: the heavy launch only zeroes the previous status set
    HIP_TRY(rcp_launch_heavy(&Q, kHeavyGrid, s));
    return end_exec(plan, s);
    RCP_CATCH
}

extern "C" int rcp_plan_execute_stages(rcp_plan* plan, double* d_out, uint8_t* d_valid, int64_t* d_binsum,
                                       void* hip_stream, int stages) {
    RCP_TRY
    if (!plan) return fail(RCP_EINVAL, "NULL plan");
    if (plan->dev.n_parts == 0) return fail(RCP_EINVAL, "coverage-only plan (created with bins == NULL)");
    if (!d_out && plan->n_rows && plan->n_cols) return fail(RCP_EINVAL, "NULL output");
    DeviceGuard g(plan->rs->device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (stages & RCP_STAGE_LOCATE) {
        // locate (also clears the previous execution's heavy slots and status words, and writes
        // the caller's validity vector), heavy slices; a folded plan's pileup kernel does both
        begin_exec(plan);
        if (!plan->dev.fold) {
            RcpPlanDev Q = plan->dev;
            Q.valid_out = d_valid;
            HIP_TRY(rcp_launch_locate(&Q, s));
            HIP_TRY(rcp_launch_heavy(&Q, kHeavyGrid, s));
        }
    }
    // rows with fewer positions than bins (splines of short genes: serial chains) write only their
    // own cells.  Row-wave plans with the HBM stage pile them in the pileup kernel (interp_stage:
    // the interpolation kernel, after it, reads their depth from the stage -- no second pileup of
    // the row); other plans' interpolation reads only locate's outputs and runs on a side stream
    // beside the pileup, joining the caller's stream after it
    plan->dev.interp_stage = (plan->dev.lean == 3 && plan->dev.rm32 && !d_binsum) ? 1 : 0;
    const bool fork = (stages & RCP_STAGE_PILEUP) && (stages & RCP_STAGE_INTERP) && plan->dev.n_interp > 0 &&
                      !plan->dev.interp_stage && !plan->dev.fold;  // (folded: the pileup kernel locates)
    if (fork) {
        if (!plan->side) {
            HIP_TRY(hipStreamCreateWithFlags(&plan->side, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&plan->ev_fork, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&plan->ev_join, hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(plan->ev_fork, s));
        HIP_TRY(hipStreamWaitEvent(plan->side, plan->ev_fork, 0));
        HIP_TRY(rcp_launch_interp(&plan->dev, d_out, plan->side));
        HIP_TRY(hipEventRecord(plan->ev_join, plan->side));
    }
    if (stages & RCP_STAGE_PILEUP) {
        RcpPlanDev Q = plan->dev;
        if (Q.fold) Q.valid_out = d_valid;
        HIP_TRY(rcp_launch_pileup(&Q, d_out, d_binsum, 0, s));
    }
    // (row-wave plans with the HBM stage interpolate in the pileup kernel: the wave that piled
    // the row runs its spline)
    const bool fused = plan->dev.interp_stage && plan->dev.interp_of;
    if (fork) HIP_TRY(hipStreamWaitEvent(s, plan->ev_join, 0));
    else if ((stages & RCP_STAGE_INTERP) && !fused) HIP_TRY(rcp_launch_interp(&plan->dev, d_out, s));
    return end_exec(plan, s);
    RCP_CATCH
}

extern "C" int rcp_plan_execute(rcp_plan* plan, double* d_out, uint8_t* d_valid, int64_t* d_binsum,
                                void* hip_stream) {
    RCP_TRY
    return rcp_plan_execute_stages(plan, d_out, d_valid, d_binsum, hip_stream, RCP_STAGE_ALL);
    RCP_CATCH
}

extern "C" int rcp_plan_status(rcp_plan* plan, void* hip_stream) {
    RCP_TRY
    if (!plan) return fail(RCP_EINVAL, "NULL plan");
    DeviceGuard g(plan->rs->device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    uint32_t st = 0;
    HIP_TRY(hipMemcpyAsync(&st, plan->dev.status, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (st & RCP_STATUS_WIDTH)
        return fail(RCP_EUNSUPPORTED, "a per-base part met a row whose slice width differs from the column count");
    if (st & RCP_STATUS_INTERP) return fail(RCP_EUNSUPPORTED, "internal plan/layout mismatch (status %u)", st);
    if (st & RCP_STATUS_OVERFLOW) return fail(RCP_EUNSUPPORTED, "bin numerator exceeded 2^32");
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_plan_heavy_rows(rcp_plan* plan, void* hip_stream, int32_t* n_rows) {
    RCP_TRY
    if (!plan || !n_rows) return fail(RCP_EINVAL, "NULL argument");
    DeviceGuard g(plan->rs->device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    uint32_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, plan->dev.status + 1, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_rows = (int32_t)std::min<uint32_t>(n, (uint32_t)std::max(plan->dev.heavy_cap, 0));
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_profile(const rcp_readset* rs, const rcp_rows_desc* rows, const rcp_bins_desc* bins, double* out,
                           uint8_t* row_valid) {
    RCP_TRY
    rcp_plan* plan = nullptr;
    // padded column stride on the device (whole 128-B lines per 16-row column segment); the
    // staged copy drops the padding on the way into R's n_rows x n_cols matrix
    rcp_plan_opts opts{RCP_KERNEL_AUTO, -1, RCP_OUT_LD_PADDED, 0, 0, {0, 0}};
    int rc = rcp_plan_create_ex(rs, rows, bins, &opts, &plan);
    if (rc) return rc;
    std::unique_ptr<rcp_plan, int (*)(rcp_plan*)> guard(plan, rcp_plan_destroy);
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);
    const size_t cells = (size_t)plan->out_ld * (size_t)plan->n_cols;
    DevBuf d_out, d_valid;
    HIP_TRY(d_out.alloc(8 * std::max<size_t>(cells, 1)));
    HIP_TRY(d_valid.alloc(std::max<int32_t>(plan->n_rows, 1)));
    rc = rcp_plan_execute(plan, d_out.as<double>(), d_valid.as<uint8_t>(), nullptr, nullptr);
    if (rc) return rc;
    rc = rcp_plan_status(plan, nullptr);
    if (rc) return rc;
    // into R's allocMatrix memory (pageable): pinned double-buffered staging (rcp_stage.h)
    if (out && plan->n_rows && plan->n_cols) {
        rc = download_matrix(plan, d_out.as<double>(), out, (size_t)plan->n_rows, nullptr);
        if (rc) return rc;
    }
    if (row_valid && plan->n_rows) HIP_TRY(hipMemcpy(row_valid, d_valid.p, plan->n_rows, hipMemcpyDeviceToHost));
    return RCP_OK;
    RCP_CATCH
}


extern "C" int rcp_readset_create_multi(const rcp_reads_desc* desc, const int32_t* device_ids, int32_t n_devices,
                                        rcp_readset** out) {
    RCP_TRY
    if (!desc || !device_ids || !out) return fail(RCP_EINVAL, "NULL argument");
    if (n_devices < 1 || n_devices > 64) return fail(RCP_EINVAL, "n_devices = %d", n_devices);
    for (int i = 0; i < n_devices; ++i) {
        out[i] = nullptr;
        const int rc = check_device(device_ids[i]);
        if (rc) return rc;
    }
    const int rc = run_per_device(n_devices, [&](int i) {
        rcp_reads_desc d = *desc;
        d.device = device_ids[i];
        return rcp_readset_create(&d, nullptr, &out[i]);
    });
    if (rc) {
        for (int i = 0; i < n_devices; ++i) {
            rcp_readset_destroy(out[i]);
            out[i] = nullptr;
        }
    }
    return rc;
    RCP_CATCH
}

namespace {

// One sample's reads cut for one row table (rcp_profile_reads): row block b = rows
// [rows[b], rows[b + 1]) needs only the reads [a[b], z[b]) of the caller's arrays.
struct StreamCut {
    std::vector<int32_t> rows;
    std::vector<int64_t> a, z;
};

// The cut of a sample whose host reads are coordinate-sorted -- chromosome runs, each code in
// one run, starts ascending inside a run (what a sorted BAM gives: R/ranges.R:111-132 keeps file
// order) -- and come with width runs (the widest read bounds how far before a range its reads
// start).  Row blocks of equal row count (equal matrix bytes to copy down); each block's reads
// are found by bisection of the host starts per chromosome, and the slices together cover every
// read, so that the device check of each slice (kLayCheckOrder) plus the host check of the pair
// in front of every slice end prove the order the bisections assumed.  false: the sample goes
// as one piece (per-read chromosome or end vectors, few reads or rows, or slices that would
// overlap much -- rows in another chromosome order than the reads).
bool stream_cut(const rcp_reads_desc& d, const rcp_rows_desc* rows, StreamCut* cut) {
    const int64_t n = d.n;
    const int32_t R = rows->n_rows;
    if (d.on_device || d.chrom || d.end || !d.start || n < (int64_t(1) << 22) || R < 2048) return false;
    if (d.n_chrom_runs <= 0 || !d.chrom_run_value || !d.chrom_run_length || d.n_width_runs <= 0 ||
        !d.width_run_value || !d.width_run_length || d.n_chrom <= 0)
        return false;
    int32_t maxw = 0;
    for (int32_t k = 0; k < d.n_width_runs; ++k) {
        if (d.width_run_value[k] < 0) return false;  // (the build reports it)
        maxw = std::max(maxw, d.width_run_value[k]);
    }
    // chromosome code -> its run [cs, ce)
    std::vector<int64_t> cs(d.n_chrom, -1), ce(d.n_chrom, -1), run_at;
    run_at.reserve(d.n_chrom_runs + 1);
    int64_t pos = 0;
    for (int32_t k = 0; k < d.n_chrom_runs; ++k) {
        const int32_t c = d.chrom_run_value[k];
        if (d.chrom_run_length[k] <= 0) return false;
        if (c >= 0 && c < d.n_chrom) {
            if (cs[c] >= 0) return false;  // a chromosome in two runs: not grouped
            cs[c] = pos;
            ce[c] = pos + d.chrom_run_length[k];
        }
        run_at.push_back(pos);
        pos += d.chrom_run_length[k];
    }
    if (pos != n) return false;
    const int nb = (int)std::min<int64_t>(8, std::max<int64_t>(2, n >> 22));  // >= 4 M reads a block
    // the first blocks smaller (a quarter, three quarters of the others): the first rows of the
    // matrix start down sooner, and the download -- the longer direction -- runs longer
    std::vector<double> w(nb, 1.0);
    if (nb >= 4) {
        w[0] = 0.25;
        w[1] = 0.75;
    }
    double wsum = 0.0;
    for (double x : w) wsum += x;
    cut->rows.assign(nb + 1, 0);
    double acc = 0.0;
    for (int b = 0; b < nb; ++b) {
        acc += w[b];
        cut->rows[b + 1] = b + 1 == nb ? R : (int32_t)std::min<double>(R, std::floor(R * acc / wsum));
    }
    std::vector<int64_t> L(nb, n), H(nb, 0), smin(d.n_chrom), emax(d.n_chrom);
    std::vector<char> touched(d.n_chrom, 0);
    std::vector<int32_t> list;
    const int32_t* st = d.start;
    for (int b = 0; b < nb; ++b) {
        list.clear();
        for (int64_t j = rows->seg_off[cut->rows[b]]; j < rows->seg_off[cut->rows[b + 1]]; ++j) {
            const int32_t c = rows->seg_chrom[j];
            if (c < 0 || c >= d.n_chrom || cs[c] < 0) continue;
            const int64_t s0 = std::max<int64_t>(rows->seg_start[j], 1), e0 = rows->seg_end[j];
            if (e0 < s0) continue;
            const int64_t lo = s0 - maxw + 1;  // a read overlapping [s0, e0] starts in [lo, e0]
            if (!touched[c]) {
                touched[c] = 1;
                list.push_back(c);
                smin[c] = lo;
                emax[c] = e0;
            } else {
                smin[c] = std::min(smin[c], lo);
                emax[c] = std::max(emax[c], e0);
            }
        }
        for (int32_t c : list) {
            touched[c] = 0;
            const int64_t l = std::lower_bound(st + cs[c], st + ce[c], smin[c],
                                               [](int32_t v, int64_t x) { return (int64_t)v < x; }) - st;
            const int64_t h = std::upper_bound(st + cs[c], st + ce[c], emax[c],
                                               [](int64_t x, int32_t v) { return x < (int64_t)v; }) - st;
            if (h > l) {
                L[b] = std::min(L[b], l);
                H[b] = std::max(H[b], h);
            }
        }
    }
    // slices: [a_b, z_b) holds block b's reads; together they cover [0, n)
    cut->a.assign(nb, 0);
    cut->z.assign(nb, 0);
    int64_t Z = 0, total = 0;
    for (int b = 0; b < nb; ++b) {
        cut->a[b] = b == 0 ? 0 : std::min(L[b], Z);
        cut->z[b] = b == nb - 1 ? n : std::max(H[b], cut->a[b]);
        Z = std::max(Z, cut->z[b]);
        total += cut->z[b] - cut->a[b];
    }
    if (total > n + n / 4) return false;
    // the pair of reads in front of each slice end (the device checks the pairs inside a slice)
    for (int b = 0; b < nb; ++b) {
        const int64_t i = cut->z[b];
        if (i <= 0 || i >= n) continue;
        const bool same_run = !std::binary_search(run_at.begin(), run_at.end(), i);
        if (same_run && st[i - 1] > st[i]) return false;
    }
    return true;
}

}  // namespace

extern "C" int rcp_profile_reads(const rcp_reads_desc* samples, int32_t n_samples, const rcp_rows_desc* rows,
                                 const rcp_bins_desc* bins, double* const* outs, uint8_t* const* row_valid) {
    RCP_TRY
    if (!samples || !rows || !bins) return fail(RCP_EINVAL, "NULL argument");
    if (n_samples < 0) return fail(RCP_EINVAL, "n_samples = %d", n_samples);
    if (n_samples == 0) return RCP_OK;
    const int dev = samples[0].device;
    for (int i = 0; i < n_samples; ++i)
        if (samples[i].device != dev)
            return fail(RCP_EINVAL, "samples[%d] is for device %d, samples[0] for %d (one device per call)", i,
                        samples[i].device, dev);
    int rc = check_device(dev);
    if (rc) return rc;
    // every descriptor checked before anything is cut or copied (stream_cut indexes the row table,
    // the packed uploads read the strand arrays)
    rc = validate_rows(rows);
    if (rc) return rc;
    for (int i = 0; i < n_samples; ++i)
        if ((rc = validate_reads(&samples[i]))) {
            const std::string msg = rcp_last_error();
            return fail(rc, "samples[%d]: %s", i, msg.c_str());
        }
    const int32_t R = rows->n_rows;
    // the one layout the row table searches, built from the uploaded copies right away
    const int layout = rows->ignore_strand ? kLayMerged : kLayStranded;
    // Work items: a sample of sorted reads is cut into row blocks, each with the slice of the
    // reads it needs (stream_cut); any other sample is one item.  Four host threads:
    //   uploader  -- copies each block's slice of starts and strands up (the upload staging
    //                buffers) into device buffers, at most two slices ahead of the builder;
    //   builder   -- builds each block's readset from its device slice (order check, sort, index);
    //                a whole item's readset straight from the host arrays;
    //   profilers -- two, taking the built items in order: plan, pass, and the block's rows of
    //                the matrix copied down (the download staging buffers) -- while one copies
    //                down, the other plans and runs.
    // Both PCIe directions stay busy; the uploads run ahead (three slices up, four readsets alive)
    // so that they end early and the longer download then has the link to itself.  A sample whose
    // slices prove unsorted on the device is redone as one item after its blocks in flight.
    struct Staged {
        int sample;
        int32_t r0, r1;
        bool whole;
        ReadSlice sl;
        void* d_start;
        void* d_strand;
    };
    struct Item {
        int sample;
        int32_t r0, r1;
        bool redo;
        rcp_readset* rs;
    };
    std::deque<Staged> staged;
    int n_staged = 0;  // slices up, not yet taken by the builder
    std::deque<Item> items;
    size_t next = 0;
    int alive = 0;
    bool up_done = false, built_done = false, abort = false;
    std::vector<char> poisoned(n_samples, 0);
    std::vector<int> active(n_samples, 0);
    std::mutex mu;
    std::condition_variable cv;
    const bool tr = rcp::trace_on();
    const double t0 = tr ? rcp::trace_ms() : 0.0;
    auto set_abort = [&] {
        {
            std::lock_guard<std::mutex> lock(mu);
            abort = true;
        }
        cv.notify_all();
    };
    const int r2 = run_per_device(4, [&](int role) -> int {
        DeviceGuard g(dev);
        HIP_TRY(g.err);
        hipStream_t s = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        std::unique_ptr<std::remove_pointer<hipStream_t>::type, hipError_t (*)(hipStream_t)> sguard(s, hipStreamDestroy);
        if (role == 0) {  // uploader
            auto push = [&](Staged&& x) {
                {
                    std::lock_guard<std::mutex> lock(mu);
                    if (!x.whole) ++n_staged;
                    staged.push_back(std::move(x));
                }
                cv.notify_all();
            };
            for (int k = 0; k < n_samples; ++k) {
                StreamCut cut;
                if (!stream_cut(samples[k], rows, &cut)) {
                    push(Staged{k, 0, R, true, {}, nullptr, nullptr});
                    continue;
                }
                for (size_t b = 0; b + 1 < cut.rows.size(); ++b) {
                    {
                        std::unique_lock<std::mutex> lock(mu);
                        cv.wait(lock, [&] { return abort || n_staged < 3 || poisoned[k]; });
                        if (abort) return (int)RCP_OK;
                        if (poisoned[k]) break;
                    }
                    Staged x{k, cut.rows[b], cut.rows[b + 1], false, {}, nullptr, nullptr};
                    slice_reads(&samples[k], cut.a[b], cut.z[b], &x.sl);
                    const int64_t n = x.sl.d.n;
                    const double tb = tr ? rcp::trace_ms() : 0.0;
                    hipError_t e = hipSuccess;
                    if (n > 0) {
                        e = pool_alloc(&x.d_start, 4 * (size_t)n, s);
                        if (e == hipSuccess) e = pool_alloc(&x.d_strand, (size_t)n, s);
                        if (e == hipSuccess)
                            e = rcp::stage_h2d_i32(static_cast<int32_t*>(x.d_start), x.sl.d.start, (size_t)n, dev, s);
                        if (e == hipSuccess)
                            e = rcp::stage_h2d_strand(static_cast<int8_t*>(x.d_strand), x.sl.d.strand, (size_t)n, dev, s);
                    }
                    if (tr)
                        fprintf(stderr, "[reads] sample %d block %zu: %lld reads up %.2f ms (at %.2f)\n", k, b,
                                (long long)n, rcp::trace_ms() - tb, tb - t0);
                    if (e != hipSuccess) {
                        pool_free(x.d_start, s);
                        pool_free(x.d_strand, s);
                        set_abort();
                        HIP_TRY(e);
                    }
                    push(std::move(x));
                }
            }
            {
                std::lock_guard<std::mutex> lock(mu);
                up_done = true;
            }
            cv.notify_all();
            return (int)RCP_OK;
        }
        if (role == 1) {  // builder
            auto publish = [&](const Item& it) {
                {
                    std::lock_guard<std::mutex> lock(mu);
                    items.push_back(it);
                }
                cv.notify_all();
            };
            auto take_slot = [&]() {
                std::unique_lock<std::mutex> lock(mu);
                cv.wait(lock, [&] { return abort || alive < 4; });
                if (abort) return false;
                ++alive;
                return true;
            };
            auto drop_slot = [&] {
                std::lock_guard<std::mutex> lock(mu);
                --alive;
            };
            for (;;) {
                Staged x;
                {
                    std::unique_lock<std::mutex> lock(mu);
                    cv.wait(lock, [&] { return abort || !staged.empty() || up_done; });
                    if (abort) return (int)RCP_OK;
                    if (staged.empty()) {
                        built_done = true;
                        break;
                    }
                    x = std::move(staged.front());
                    staged.pop_front();
                    if (!x.whole) --n_staged;
                }
                cv.notify_all();
                const int k = x.sample;
                bool whole = x.whole;
                if (!whole) {
                    bool skip;
                    {
                        std::lock_guard<std::mutex> lock(mu);
                        skip = poisoned[k] != 0;
                    }
                    if (skip) {  // a slice of a sample being redone whole
                        pool_free(x.d_start, s);
                        pool_free(x.d_strand, s);
                        continue;
                    }
                    if (!take_slot()) {
                        pool_free(x.d_start, s);
                        pool_free(x.d_strand, s);
                        return (int)RCP_OK;
                    }
                    rcp_reads_desc d = x.sl.d;
                    d.on_device = 1;
                    d.start = static_cast<const int32_t*>(x.d_start);
                    d.strand = static_cast<const int8_t*>(x.d_strand);
                    rcp_readset* r = nullptr;
                    const double tb = tr ? rcp::trace_ms() : 0.0;
                    const int e = readset_build(&d, s, layout | kLayCheckOrder, &r);
                    pool_free(x.d_start, s);
                    pool_free(x.d_strand, s);
                    if (tr)
                        fprintf(stderr, "[reads] sample %d rows [%d, %d): built %.2f ms (at %.2f)\n", k, x.r0, x.r1,
                                rcp::trace_ms() - tb, tb - t0);
                    if (e == kNotInOrder) {
                        drop_slot();
                        {
                            std::lock_guard<std::mutex> lock(mu);
                            poisoned[k] = 1;
                        }
                        cv.notify_all();
                        whole = true;
                    } else if (e) {
                        drop_slot();
                        set_abort();
                        return e;
                    } else {
                        publish(Item{k, x.r0, x.r1, false, r});
                    }
                }
                if (whole) {
                    if (!take_slot()) return (int)RCP_OK;
                    rcp_readset* r = nullptr;
                    const int e = readset_build(&samples[k], s, layout, &r);
                    if (e) {
                        drop_slot();
                        set_abort();
                        return e;
                    }
                    bool redo;
                    {
                        std::lock_guard<std::mutex> lock(mu);
                        redo = poisoned[k] != 0;
                    }
                    publish(Item{k, 0, R, redo, r});
                }
            }
            cv.notify_all();
            return (int)RCP_OK;
        }
        for (;;) {  // profilers
            Item it{};
            {
                std::unique_lock<std::mutex> lock(mu);
                cv.wait(lock, [&] { return abort || next < items.size() || built_done; });
                if (abort || next >= items.size()) return (int)RCP_OK;
                it = items[next++];
                if (poisoned[it.sample] && !it.redo) {  // a block of a sample being redone whole
                    lock.unlock();
                    rcp_readset_destroy(it.rs);
                    lock.lock();
                    --alive;
                    cv.notify_all();
                    continue;
                }
                if (it.redo) cv.wait(lock, [&] { return abort || active[it.sample] == 0; });
                ++active[it.sample];
            }
            const double tb = tr ? rcp::trace_ms() : 0.0;
            rcp_rows_desc sub = *rows;
            sub.n_rows = it.r1 - it.r0;
            sub.seg_off = rows->seg_off + it.r0;
            int64_t nc = 0;
            int e = abort ? (int)RCP_OK
                          : profile_block(it.rs, &sub, bins, outs ? outs[it.sample] : nullptr, R, it.r0,
                                          row_valid ? row_valid[it.sample] : nullptr, &nc, s);
            if (tr)
                fprintf(stderr, "[reads] sample %d rows [%d, %d): profile + down %.2f ms (at %.2f)\n", it.sample, it.r0,
                        it.r1, rcp::trace_ms() - tb, tb - t0);
            rcp_readset_destroy(it.rs);  // (a device synchronisation: outside the lock)
            {
                std::lock_guard<std::mutex> lock(mu);
                --alive;
                --active[it.sample];
                if (e) abort = true;
            }
            cv.notify_all();
            if (e) return e;
        }
    });
    for (Staged& x : staged) {  // (left behind by a failure: slices not built)
        pool_free(x.d_start, nullptr);
        pool_free(x.d_strand, nullptr);
    }
    // (left behind by a failure: items not taken)
    for (size_t i = next; i < items.size(); ++i) rcp_readset_destroy(items[i].rs);
    return r2;
    RCP_CATCH
}

extern "C" int rcp_profile_samples(rcp_readset* const* readsets, int32_t n_samples, const rcp_rows_desc* rows,
                                   const rcp_bins_desc* bins, int32_t inflight, double* const* outs,
                                   uint8_t* const* row_valid) {
    RCP_TRY
    if (!readsets || !rows || !bins) return fail(RCP_EINVAL, "NULL argument");
    if (n_samples < 0) return fail(RCP_EINVAL, "n_samples = %d", n_samples);
    if (inflight < 0 || inflight > 3) return fail(RCP_EINVAL, "inflight = %d (0..3)", inflight);
    if (n_samples == 0) return RCP_OK;
    for (int i = 0; i < n_samples; ++i) {
        if (!readsets[i]) return fail(RCP_EINVAL, "readsets[%d] is NULL", i);
        if (readsets[i]->device != readsets[0]->device)
            return fail(RCP_EINVAL, "readsets[%d] is on device %d, readsets[0] on %d (one device per call)", i,
                        readsets[i]->device, readsets[0]->device);
    }
    const int dev = readsets[0]->device;
    const int D = std::min(n_samples, inflight == 0 ? 2 : inflight);
    // plans first (host work and small uploads), so the passes below are launches only
    std::vector<std::unique_ptr<rcp_plan, int (*)(rcp_plan*)>> plans;
    plans.reserve(n_samples);
    for (int i = 0; i < n_samples; ++i) {
        rcp_plan* plan = nullptr;
        rcp_plan_opts opts{RCP_KERNEL_AUTO, -1, RCP_OUT_LD_PADDED, 0, D, {0, 0}};  // D passes in flight
        const int e = rcp_plan_create_ex(readsets[i], rows, bins, &opts, &plan);
        if (e) return e;
        plans.emplace_back(plan, rcp_plan_destroy);
    }
    DeviceGuard g(dev);
    HIP_TRY(g.err);
    const rcp_plan* p0 = plans[0].get();
    const size_t cells = (size_t)p0->out_ld * (size_t)p0->n_cols;
    std::vector<DevBuf> d_out(D), d_valid(D);
    std::vector<hipStream_t> st(D, nullptr);
    struct Streams {
        std::vector<hipStream_t>& v;
        ~Streams() {
            for (hipStream_t x : v)
                if (x) (void)hipStreamDestroy(x);
        }
    } sguard{st};
    for (int k = 0; k < D; ++k) {
        HIP_TRY(d_out[k].alloc(8 * std::max<size_t>(cells, 1)));
        HIP_TRY(d_valid[k].alloc(std::max<int32_t>(p0->n_rows, 1)));
        HIP_TRY(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
    }
    // sample j's pass ran on slot j % D: wait for it, check its status, copy its matrix out
    auto finish = [&](int j) -> int {
        const int k = j % D;
        rcp_plan* plan = plans[j].get();
        int e = rcp_plan_status(plan, st[k]);
        if (e) return e;
        if (outs && outs[j] && plan->n_rows && plan->n_cols) {
            e = download_matrix(plan, d_out[k].as<double>(), outs[j], (size_t)plan->n_rows, st[k]);
            if (e) return e;
        }
        if (row_valid && row_valid[j] && plan->n_rows) {
            HIP_TRY(hipMemcpyAsync(row_valid[j], d_valid[k].p, plan->n_rows, hipMemcpyDeviceToHost, st[k]));
            HIP_TRY(hipStreamSynchronize(st[k]));
        }
        return RCP_OK;
    };
    for (int i = 0; i < n_samples; ++i) {
        if (i >= D) {
            const int e = finish(i - D);  // frees slot i % D
            if (e) return e;
        }
        const int k = i % D;
        const int e = rcp_plan_execute(plans[i].get(), d_out[k].as<double>(), d_valid[k].as<uint8_t>(), nullptr, st[k]);
        if (e) return e;
    }
    for (int j = std::max(0, n_samples - D); j < n_samples; ++j) {
        const int e = finish(j);
        if (e) return e;
    }
    return RCP_OK;
    RCP_CATCH
}

namespace rcpi {

// A plan's matrix (d_out, column stride plan->out_ld, on stream s) into the host's column-major
// double matrix (column stride host_ld): as uint32 bin numerators, 4 bytes a cell over PCIe, when
// every mean is one (rcp_pack_kernel: one-part plans without interpolated rows or R-RNG layouts,
// positive scale), the host making each double with the device's operations -- else as the
// doubles.  (C4's 1.6 GB matrix: 0.8 GB down, and 2.4 instead of 3.2 GB of host memory traffic
// -- DMA in, pinned read, destination write -- which is what bounds a streamed call.)
int download_packed(const double* d_out, size_t ld, size_t R, size_t C, double scale, double* host, size_t host_ld,
                    int device, hipStream_t s,
                    const std::function<hipError_t(uint32_t* q, uint32_t* div, uint32_t* bad_row)>& pack,
                    const std::vector<RowRun>* runs) {
    const std::vector<RowRun> all{RowRun{0, 0, R}};
    if (!runs) runs = &all;
    // the doubles of every run, straight into their host rows
    auto doubles = [&]() -> int {
        for (const RowRun& u : *runs)
            HIP_TRY(rcp::stage_d2h_2d(host + u.dst, 8 * host_ld, d_out + u.src, 8 * ld, 8 * u.len, C, device, s));
        return (int)RCP_OK;
    };
    PoolBuf q(s), aux(s);
    HIP_TRY(q.alloc(4 * ld * C));
    HIP_TRY(aux.alloc(8 * R));
    uint32_t* d_div = aux.as<uint32_t>();
    uint32_t* d_bad = d_div + R;
    HIP_TRY(hipMemsetAsync(d_bad, 0, 4 * R, s));
    HIP_TRY(pack(q.as<uint32_t>(), d_div, d_bad));
    std::vector<uint32_t> h(2 * R);
    HIP_TRY(hipMemcpyAsync(h.data(), d_div, 8 * R, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> bad;
    for (size_t r = 0; r < R; ++r)
        if (h[R + r]) bad.push_back((int32_t)r);
    // many rows the numerators cannot carry (interpolated genes, R-RNG layouts): all doubles
    if (bad.size() > R / 8) {
        if (rcp::trace_on()) fprintf(stderr, "[pack] doubles: %zu of %zu rows not numerators\n", bad.size(), R);
        return doubles();
    }
    std::vector<size_t> dst_of;  // host row of each device row (the marked rows' doubles below)
    if (runs != &all && !bad.empty()) {
        dst_of.assign(R, 0);
        for (const RowRun& u : *runs)
            for (size_t i = 0; i < u.len; ++i) dst_of[u.src + i] = u.dst + i;
    }
    for (const RowRun& u : *runs) {
        bool no_buffers = false;
        HIP_TRY(rcp::stage_d2h_expand(host + u.dst, host_ld, q.as<uint32_t>() + u.src, ld, u.len, C, h.data() + u.src,
                                      scale, device, s, &no_buffers));
        if (no_buffers) return doubles();  // no pinned buffers for this device: the doubles, as a direct copy
    }
    if (!bad.empty()) {  // those rows' doubles, gathered on the device, over the expanded cells
        const size_t nb = bad.size();
        PoolBuf d_rows(s), d_vals(s);
        HIP_TRY(d_rows.alloc(4 * nb));
        HIP_TRY(d_vals.alloc(8 * nb * C));
        HIP_TRY(hipMemcpyAsync(d_rows.p, bad.data(), 4 * nb, hipMemcpyHostToDevice, s));
        HIP_TRY(rcp_launch_gather_rows(d_out, (int64_t)ld, d_rows.as<int32_t>(), (int32_t)nb, (int64_t)C,
                                       d_vals.as<double>(), s));
        std::vector<double> vals(nb * C);
        HIP_TRY(hipMemcpyAsync(vals.data(), d_vals.p, 8 * nb * C, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (size_t c = 0; c < C; ++c)
            for (size_t i = 0; i < nb; ++i)
                host[c * host_ld + (dst_of.empty() ? (size_t)bad[i] : dst_of[(size_t)bad[i]])] = vals[c * nb + i];
        if (rcp::trace_on()) fprintf(stderr, "[pack] %zu rows as doubles\n", nb);
    }
    return RCP_OK;
}

// A plan's matrix (d_out, column stride plan->out_ld, on stream s) into the host's column-major
// double matrix (column stride host_ld): as uint32 bin numerators, 4 bytes a cell over PCIe
// (rcp_pack_kernel: one-part plans of mean bins, positive scale), the host making each double with
// the device's operations; rows the numerators cannot carry (interpolated, R-RNG layouts) come down
// apart as doubles.  Plans of several parts, or many such rows: the doubles.  (C4's 1.6 GB matrix: 0.8 GB down, and
// 2.4 instead of 3.2 GB of host memory traffic -- DMA in, pinned read, destination write --
// which is what bounds a streamed call.)
int download_matrix(rcp_plan* plan, const double* d_out, double* host, size_t host_ld, hipStream_t s,
                    const std::vector<RowRun>* runs) {
    const RcpPlanDev& P = plan->dev;
    const int dev = plan->rs->device;
    const size_t R = (size_t)plan->n_rows, C = (size_t)plan->n_cols, ld = (size_t)plan->out_ld;
    if (!host || R == 0 || C == 0) return RCP_OK;
    const bool pack = P.n_parts == 1 && P.n_interp <= plan->n_rows / 8 && P.stat == 0 && P.scale > 0.0 && std::isfinite(P.scale) &&
                      C <= 65535u * 8u && 8 * R * C >= (size_t(4) << 20) && P.csr_off == nullptr;
    if (!pack) {
        if (rcp::trace_on() && 8 * R * C >= (size_t(4) << 20))
            fprintf(stderr, "[pack] doubles: plan of %d parts, %d interpolated rows\n", P.n_parts, P.n_interp);
        if (!runs) {
            HIP_TRY(rcp::stage_d2h_2d(host, 8 * host_ld, d_out, 8 * ld, 8 * R, C, dev, s));
        } else {
            for (const RowRun& u : *runs)
                HIP_TRY(rcp::stage_d2h_2d(host + u.dst, 8 * host_ld, d_out + u.src, 8 * ld, 8 * u.len, C, dev, s));
        }
        return RCP_OK;
    }
    return download_packed(d_out, ld, R, C, P.scale, host, host_ld, dev, s,
                           [&](uint32_t* q, uint32_t* div, uint32_t* bad) {
                               return rcp_launch_pack(&P, d_out, q, div, bad, s);
                           },
                           runs);
}

int profile_block(const rcp_readset* rs, const rcp_rows_desc* sub, const rcp_bins_desc* bins, double* out,
                  int64_t n_rows_total, int32_t r0, uint8_t* row_valid, int64_t* n_cols, hipStream_t stream,
                  const int32_t* dst_rows) {
    const bool tr = rcp::trace_on();
    const double t0 = tr ? rcp::trace_ms() : 0.0;
    rcp_plan* plan = nullptr;
    rcp_plan_opts opts{RCP_KERNEL_AUTO, -1, RCP_OUT_LD_PADDED, 0, 0, {0, 0}};
    int e = rcp_plan_create_ex(rs, sub, bins, &opts, &plan);
    if (e) return e;
    std::unique_ptr<rcp_plan, int (*)(rcp_plan*)> guard(plan, rcp_plan_destroy);
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);
    if (n_cols) *n_cols = plan->n_cols;
    const double t1 = tr ? rcp::trace_ms() : 0.0;
    hipStream_t s = stream;
    if (!stream) HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::unique_ptr<std::remove_pointer<hipStream_t>::type, hipError_t (*)(hipStream_t)> sguard(
        stream ? nullptr : s, hipStreamDestroy);
    // stream-ordered from the pool: no hipMalloc / hipFree (a device-wide synchronisation that would
    // wait for other threads' uploads) per block
    const size_t cells = (size_t)plan->out_ld * (size_t)plan->n_cols;
    PoolBuf d_out(s), d_valid(s);
    HIP_TRY(d_out.alloc(8 * std::max<size_t>(cells, 1)));
    HIP_TRY(d_valid.alloc(std::max<int32_t>(plan->n_rows, 1)));
    e = rcp_plan_execute(plan, d_out.as<double>(), d_valid.as<uint8_t>(), nullptr, s);
    if (e) return e;
    e = rcp_plan_status(plan, s);
    if (e) return e;
    const double t2 = tr ? rcp::trace_ms() : 0.0;
    const size_t n = (size_t)plan->n_rows, C = (size_t)plan->n_cols;
    // the block's rows as runs of consecutive caller rows (one run: rows r0 .. in order)
    std::vector<RowRun> runs;
    if (!dst_rows) {
        runs.push_back(RowRun{0, (size_t)r0, n});
    } else {
        for (size_t i = 0; i < n; ++i) {
            if (!runs.empty() && (size_t)dst_rows[i] == runs.back().dst + runs.back().len) ++runs.back().len;
            else runs.push_back(RowRun{i, (size_t)dst_rows[i], 1});
        }
    }
    // this block's rows of every column of the caller's R matrix: run by run when the runs are few
    // and long, else (rows of a table in no particular order) through a host matrix of the block
    // whose rows the threads scatter
    const bool scatter = runs.size() > std::max<size_t>(16, n / 256);
    if (out && C && n) {
        if (!scatter) {
            e = download_matrix(plan, d_out.as<double>(), out, (size_t)n_rows_total, s, &runs);
            if (e) return e;
        } else {
            std::vector<double> tmp(n * C);
            e = download_matrix(plan, d_out.as<double>(), tmp.data(), n, s);
            if (e) return e;
            const int nt = (int)std::min<size_t>(8, std::max<size_t>(1, C / 64));
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    for (size_t c = C * t / nt; c < C * (t + 1) / nt; ++c)
                        for (const RowRun& u : runs)
                            std::memcpy(out + c * (size_t)n_rows_total + u.dst, tmp.data() + c * n + u.src, 8 * u.len);
                });
            for (auto& x : th) x.join();
        }
    }
    if (tr)
        fprintf(stderr, "[block] rows [%d, %d) in %zu runs: plan %.2f ms, pass %.2f ms, down %.2f ms\n", r0,
                r0 + plan->n_rows, runs.size(), t1 - t0, t2 - t1, rcp::trace_ms() - t2);
    if (row_valid && n) {
        std::vector<uint8_t> v(n);
        HIP_TRY(hipMemcpyAsync(v.data(), d_valid.p, n, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (const RowRun& u : runs) std::memcpy(row_valid + u.dst, v.data() + u.src, u.len);
    }
    return RCP_OK;
}

// Contiguous row blocks [split[i], split[i + 1]) of near-equal total weight (cum: prefix sums
// of the per-row weights, n_rows + 1 entries)
std::vector<int32_t> balanced_split(const std::vector<double>& cum, int32_t n_blocks) {
    const int32_t R = (int32_t)cum.size() - 1;
    std::vector<int32_t> split(n_blocks + 1, 0);
    split[n_blocks] = R;
    for (int i = 1; i < n_blocks; ++i) {
        const double target = cum[R] * i / n_blocks;
        split[i] = (int32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        split[i] = std::min(std::max(split[i], split[i - 1]), R);
    }
    return split;
}

}  // namespace rcpi

extern "C" int rcp_profile_multi(rcp_readset* const* readsets, int32_t n_devices, const rcp_rows_desc* rows,
                                 const rcp_bins_desc* bins, double* out, uint8_t* row_valid, int32_t* row_split) {
    RCP_TRY
    if (!readsets || !rows || !bins) return fail(RCP_EINVAL, "NULL argument");
    if (n_devices < 1 || n_devices > 64) return fail(RCP_EINVAL, "n_devices = %d", n_devices);
    for (int i = 0; i < n_devices; ++i)
        if (!readsets[i]) return fail(RCP_EINVAL, "readsets[%d] is NULL", i);
    const int32_t R = rows->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && (!rows->seg_off || !rows->seg_chrom || !rows->seg_start || !rows->seg_end || !rows->seg_strand))
        return fail(RCP_EINVAL, "NULL row array");
    // contiguous row blocks balanced by each row's candidate reads, counted on the first device
    // (the reads a row's pileup streams), plus its length / 8 and a constant (its output and
    // per-row work): a count, not the genomic width, so hot peaks weigh what they cost
    std::vector<int32_t> split(n_devices + 1, 0);
    split[n_devices] = R;
    if (n_devices > 1 && R > 0) {
        std::vector<uint2> b;
        const int e = seg_bounds(readsets[0], rows, &b);
        if (e) return e;
        std::vector<double> cum(R + 1, 0.0);
        for (int32_t r = 0; r < R; ++r) {
            double w = 16.0;
            for (int64_t j = rows->seg_off[r]; j < rows->seg_off[r + 1]; ++j) {
                for (int k = 0; k < 3; ++k) w += (double)(b[3 * j + k].y - b[3 * j + k].x);
                w += std::max<double>(0.0, (double)rows->seg_end[j] - rows->seg_start[j] + 1) / 8.0;
            }
            cum[r + 1] = cum[r] + w;
        }
        split = balanced_split(cum, n_devices);
    }
    if (row_split) std::copy(split.begin(), split.end(), row_split);
    std::vector<int64_t> n_cols(n_devices, -1);
    const int rc = run_per_device(n_devices, [&](int i) {
        const int32_t r0 = split[i], r1 = split[i + 1];
        if (r1 <= r0) return (int)RCP_OK;
        rcp_rows_desc sub = *rows;  // seg_off indexes the shared segment arrays directly
        sub.n_rows = r1 - r0;
        sub.seg_off = rows->seg_off + r0;
        return profile_block(readsets[i], &sub, bins, out, R, r0, row_valid, &n_cols[i]);
    });
    if (rc) return rc;
    int64_t nc = -1;
    for (int i = 0; i < n_devices; ++i) {
        if (n_cols[i] < 0) continue;
        if (nc >= 0 && n_cols[i] != nc) return fail(RCP_EINVAL, "row blocks disagree on the column count");
        nc = n_cols[i];
    }
    return RCP_OK;
    RCP_CATCH
}

namespace {

// calcCoverage of every row into CSR depth (d_off: device [n_rows + 1])
int calc_coverage_dev(rcp_plan* plan, const int64_t* d_off, int32_t* d_cov, uint8_t* d_valid, hipStream_t s) {
    // one per-base part over the whole row, chunked by the plan's chunk capacity
    begin_exec(plan);
    RcpPlanDev P = plan->dev;
    P.n_parts = 1;
    RcpPart& pt = P.part[0];
    pt = RcpPart{};
    pt.hi_end = 1;
    pt.per_base = 1;
    pt.n_bins = std::max<int32_t>(plan->max_row_len, 1);
    pt.chunk_bins = std::max<int32_t>(std::min(P.chunk_cap, pt.n_bins), 1);
    pt.n_chunks = (pt.n_bins + pt.chunk_bins - 1) / pt.chunk_bins;
    P.n_chunks_total = pt.n_chunks;
    P.crange = nullptr;  // sized for the plan's chunks, not these
    P.cw_len = -1;
    P.lean = 0;  // the general kernel's CSR mode (locate writes every side output)
    P.fold = 0;
    P.csr_off = d_off;
    P.csr_out = d_cov;
    P.valid_out = d_valid;
    P.csr_rs = nullptr;
    HIP_TRY(rcp_launch_locate(&P, s));
    HIP_TRY(rcp_launch_heavy(&P, kHeavyGrid, s));
    HIP_TRY(rcp_launch_pileup(&P, nullptr, nullptr, 1, s));
    return end_exec(plan, s);
}

// calcCoverage of every row as run-start lists (no dense depth): per (row, column chunk of
// *chunk positions) the chunk's run starts at d_rs + d_off[row] + first position and
// (starts, last depth) at d_sub[d_sub_off[row] + chunk]
int coverage_starts_dev(rcp_plan* plan, const int64_t* d_off, const int64_t* d_sub_off, int2* d_rs, int2* d_sub,
                        uint8_t* d_valid, hipStream_t s) {
    begin_exec(plan);
    RcpPlanDev P = plan->dev;
    P.n_parts = 1;
    RcpPart& pt = P.part[0];
    pt = RcpPart{};
    pt.hi_end = 1;
    pt.per_base = 1;
    pt.n_bins = std::max<int32_t>(plan->max_row_len, 1);
    pt.chunk_bins = std::max<int32_t>(std::min(P.chunk_cap, pt.n_bins), 1);
    pt.n_chunks = (pt.n_bins + pt.chunk_bins - 1) / pt.chunk_bins;
    P.n_chunks_total = pt.n_chunks;
    P.crange = nullptr;
    P.cw_len = -1;
    P.lean = 0;
    P.fold = 0;
    // four rounds of 16 rows per workgroup (C4 coverage pileup 632 -> 601 us vs two, 635 with
    // one; profiles/r04/r4x)
    {
        int tile = 16, rmax = 4;
        rcp_tile_geometry(&tile, &rmax);
        P.rounds = std::min(rmax, 4);
        // (fewer rounds when that leaves fewer than two workgroups per CU)
        while (P.rounds > 1 && (int64_t)((P.n_rows + tile * P.rounds - 1) / (tile * P.rounds)) * P.n_chunks_total <
                                   2 * (int64_t)std::max(P.n_cus, 1))
            P.rounds /= 2;
    }
    P.csr_off = d_off;
    P.csr_out = nullptr;
    P.valid_out = d_valid;
    P.csr_rs = d_rs;
    P.csr_sub = d_sub;
    P.csr_sub_off = d_sub_off;
    HIP_TRY(rcp_launch_locate(&P, s));
    HIP_TRY(rcp_launch_heavy(&P, kHeavyGrid, s));
    HIP_TRY(rcp_launch_pileup(&P, nullptr, nullptr, 1, s));
    return end_exec(plan, s);
}

// the column chunk of coverage_starts_dev (one wave sub-chunk each)
int32_t coverage_chunk(const rcp_plan* plan) {
    return std::max<int32_t>(std::min(plan->dev.chunk_cap, std::max<int32_t>(plan->max_row_len, 1)), 1);
}

}  // namespace


extern "C" int rcp_calc_coverage(rcp_plan* plan, const int64_t* out_off, int32_t* d_cov, uint8_t* d_valid,
                                 void* hip_stream) {
    RCP_TRY
    if (!plan || !out_off) return fail(RCP_EINVAL, "NULL argument");
    DeviceGuard g(plan->rs->device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    for (int r = 0; r < plan->n_rows; ++r)
        if (out_off[r + 1] - out_off[r] != plan->row_len[r])
            return fail(RCP_EINVAL, "out_off does not match the row lengths at row %d", r);
    DevBuf d_off;
    HIP_TRY(d_off.alloc(8 * (plan->n_rows + 1)));
    HIP_TRY(hipMemcpyAsync(d_off.p, out_off, 8 * (plan->n_rows + 1), hipMemcpyHostToDevice, s));
    const int rc = calc_coverage_dev(plan, d_off.as<int64_t>(), d_cov, d_valid, s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));  // d_off is released on return
    return RCP_OK;
    RCP_CATCH
}

namespace {

// Run-length encoding of CSR coverage on the device (rcp_kernels.hip: count, scan, emit).
// d_run_off: device [n_rows + 1]; the total run count is returned in *n_runs (one sync).
// d_values / d_lengths: device arrays of at least n_runs entries, or null to only count
// (then call again with them).
int rle_encode_device(int32_t n_rows, const int64_t* d_off, const int32_t* d_cov, int64_t* d_run_off,
                      int64_t* n_runs, hipStream_t s) {
    PoolBuf count(s), temp(s);
    HIP_TRY(count.alloc(8 * ((size_t)n_rows + 1)));
    size_t tb = 0;
    HIP_TRY(rcp_rle_encode_dev(n_rows, d_off, d_cov, count.as<int64_t>(), d_run_off, nullptr, &tb, nullptr, nullptr, 0,
                               s));
    HIP_TRY(temp.alloc(std::max<size_t>(tb, 1)));
    HIP_TRY(rcp_rle_encode_dev(n_rows, d_off, d_cov, count.as<int64_t>(), d_run_off, temp.p, &tb, nullptr, nullptr, 1,
                               s));
    int64_t nr = 0;
    HIP_TRY(hipMemcpyAsync(&nr, d_run_off + n_rows, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_runs = nr;
    return RCP_OK;
}

}  // namespace

extern "C" int rcp_rle_encode(int32_t n_rows, const int64_t* out_off, const int32_t* d_cov, int device,
                              int32_t* d_values, int32_t* d_lengths, int64_t* run_off, int64_t* n_runs,
                              void* hip_stream) {
    RCP_TRY
    if (n_rows < 0 || !out_off || !run_off || !n_runs) return fail(RCP_EINVAL, "NULL argument");
    const int64_t n = out_off[n_rows];
    if (n < 0 || n >= (int64_t(1) << 31)) return fail(RCP_EUNSUPPORTED, "%lld positions", (long long)n);
    if (n > 0 && (!d_cov || !d_values || !d_lengths)) return fail(RCP_EINVAL, "NULL device array");
    if (out_off[0] != 0) return fail(RCP_EINVAL, "out_off[0] != 0");
    for (int32_t r = 0; r < n_rows; ++r)
        if (out_off[r + 1] < out_off[r]) return fail(RCP_EINVAL, "out_off decreases at row %d", r);
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    HIP_TRY(g.err);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    PoolBuf d_off(s), d_run_off(s);
    HIP_TRY(d_off.alloc(8 * ((size_t)n_rows + 1)));
    HIP_TRY(d_run_off.alloc(8 * ((size_t)n_rows + 1)));
    HIP_TRY(hipMemcpyAsync(d_off.p, out_off, 8 * ((size_t)n_rows + 1), hipMemcpyHostToDevice, s));
    int64_t nr = 0;
    rc = rle_encode_device(n_rows, d_off.as<int64_t>(), d_cov, d_run_off.as<int64_t>(), &nr, s);
    if (rc) return rc;
    PoolBuf bad(s);
    HIP_TRY(bad.alloc(4));
    HIP_TRY(hipMemsetAsync(bad.p, 0, 4, s));
    HIP_TRY(rcp_rle_encode_dev(n_rows, d_off.as<int64_t>(), d_cov, nullptr, d_run_off.as<int64_t>(), bad.p, nullptr,
                               d_values, d_lengths, 2, s));
    HIP_TRY(hipMemcpyAsync(run_off, d_run_off.p, 8 * ((size_t)n_rows + 1), hipMemcpyDeviceToHost, s));
    uint32_t h_bad = 0;
    HIP_TRY(hipMemcpyAsync(&h_bad, bad.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h_bad) return fail(RCP_EINVAL, "internal: run counts and emitted runs disagree");
    *n_runs = nr;
    return RCP_OK;
    RCP_CATCH
}

// =====================================================================================
// calcCoverage for host callers: the Rle list (what the R shim hands back).  The runs stay
// on the device until rcp_cov_copy moves them straight into the caller's arrays (R's
// allocVector results): one PCIe transfer, no library-side host copy.
// =====================================================================================

extern "C" int rcp_coverage_rle(const rcp_readset* rs, const rcp_rows_desc* rows, rcp_cov** out) {
    RCP_TRY
    if (!rs || !rows || !out) return fail(RCP_EINVAL, "NULL argument");
    *out = nullptr;
    rcp_plan* plan = nullptr;
    int rc = rcp_plan_create(rs, rows, nullptr, &plan);
    if (rc) return rc;
    std::unique_ptr<rcp_plan, int (*)(rcp_plan*)> guard(plan, rcp_plan_destroy);
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);
    const int32_t R = plan->n_rows;
    auto res = std::make_unique<rcp_cov>();
    res->n_rows = R;
    res->device = rs->device;
    std::vector<int64_t> off((size_t)R + 1, 0);
    for (int32_t r = 0; r < R; ++r) off[r + 1] = off[r] + plan->row_len[r];
    const int64_t n = off[R];
    if (n >= (int64_t(1) << 31)) return fail(RCP_EUNSUPPORTED, "%lld coverage positions", (long long)n);
    hipStream_t s = nullptr;
    {
        // the pileup writes each (row, column chunk)'s run starts (depth, position) compacted at
        // the chunk's dense offset -- no depth array --; a thread per row merges the seams
        // between chunks, a scan of the kept counts places the runs, and a wave per chunk copies
        // them out as (value, length)
        const int32_t chunk = coverage_chunk(plan);
        std::vector<int64_t> sub_off((size_t)R + 1, 0);
        for (int32_t r = 0; r < R; ++r) sub_off[r + 1] = sub_off[r] + (plan->row_len[r] + chunk - 1) / chunk;
        const int64_t S = sub_off[R];
        PoolBuf d_rs(s), d_off(s), d_sub_off(s), d_sub(s), d_cnt(s), d_info(s), d_base(s), temp(s), bad(s);
        HIP_TRY(d_rs.alloc(8 * std::max<int64_t>(n, 1)));
        HIP_TRY(d_off.alloc(8 * ((size_t)R + 1)));
        HIP_TRY(d_sub_off.alloc(8 * ((size_t)R + 1)));
        HIP_TRY(d_sub.alloc(8 * std::max<int64_t>(S, 1)));
        HIP_TRY(d_cnt.alloc(8 * ((size_t)S + 1)));
        HIP_TRY(d_info.alloc(16 * std::max<int64_t>(S, 1)));
        HIP_TRY(d_base.alloc(8 * ((size_t)S + 1)));
        HIP_TRY(bad.alloc(4));
        HIP_TRY(res->valid.alloc(std::max<int32_t>(R, 1)));
        HIP_TRY(res->run_off.alloc(8 * ((size_t)R + 1)));
        HIP_TRY(hipMemcpyAsync(d_off.p, off.data(), 8 * ((size_t)R + 1), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_sub_off.p, sub_off.data(), 8 * ((size_t)R + 1), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(d_cnt.as<int64_t>() + S, 0, 8, s));
        HIP_TRY(hipMemsetAsync(bad.p, 0, 4, s));
        rc = coverage_starts_dev(plan, d_off.as<int64_t>(), d_sub_off.as<int64_t>(), d_rs.as<int2>(), d_sub.as<int2>(),
                                 res->valid.as<uint8_t>(), s);
        if (rc) return rc;
        rc = rcp_plan_status(plan, nullptr);
        if (rc) return rc;
        size_t tb = 0;
        HIP_TRY(rcp_cov_runs_dev(R, nullptr, nullptr, S, nullptr, nullptr, nullptr, chunk, d_cnt.as<int64_t>(), nullptr,
                                 d_base.as<int64_t>(), nullptr, nullptr, &tb, nullptr, nullptr, nullptr, 0, s));
        HIP_TRY(temp.alloc(std::max<size_t>(tb, 1)));
        HIP_TRY(rcp_cov_runs_dev(R, d_off.as<int64_t>(), d_sub_off.as<int64_t>(), S, d_sub.as<int2>(), d_rs.as<int2>(),
                                 res->valid.as<uint8_t>(), chunk, d_cnt.as<int64_t>(), d_info.as<int4>(),
                                 d_base.as<int64_t>(), res->run_off.as<int64_t>(), temp.p, &tb, nullptr, nullptr,
                                 bad.as<uint32_t>(), 1, s));
        int64_t nr = 0;
        HIP_TRY(hipMemcpyAsync(&nr, res->run_off.as<int64_t>() + R, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        res->n_runs = nr;
        HIP_TRY(res->values.alloc(4 * (size_t)std::max<int64_t>(nr, 1)));
        HIP_TRY(res->lengths.alloc(4 * (size_t)std::max<int64_t>(nr, 1)));
        HIP_TRY(rcp_cov_runs_dev(R, nullptr, nullptr, S, nullptr, d_rs.as<int2>(), nullptr, chunk, nullptr,
                                 d_info.as<int4>(), d_base.as<int64_t>(), nullptr, nullptr, nullptr,
                                 res->values.as<int32_t>(), res->lengths.as<int32_t>(), bad.as<uint32_t>(), 2, s));
        uint32_t h_bad = 0;
        HIP_TRY(hipMemcpyAsync(&h_bad, bad.p, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (h_bad) return fail(RCP_EINVAL, "internal: run starts and chunk records disagree");
    }
    *out = res.release();
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_cov_info(const rcp_cov* c, int32_t* n_rows, int64_t* n_runs) {
    RCP_TRY
    if (!c) return fail(RCP_EINVAL, "NULL coverage");
    if (n_rows) *n_rows = c->n_rows;
    if (n_runs) *n_runs = c->n_runs;
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_cov_copy(const rcp_cov* c, int64_t* run_off, int32_t* values, int32_t* lengths,
                            uint8_t* valid) {
    RCP_TRY
    if (!c) return fail(RCP_EINVAL, "NULL coverage");
    if (!c->parts.empty()) return cov_copy_parts(c, run_off, values, lengths, valid);
    DeviceGuard g(c->device);
    HIP_TRY(g.err);
    // pinned double-buffered staging (rcp_stage.h) straight into the caller's arrays
    if (run_off) HIP_TRY(rcp::stage_d2h(run_off, c->run_off.p, 8 * ((size_t)c->n_rows + 1), c->device, nullptr));
    // (depths and run lengths: 16-bit offsets within blocks where they fit, rcp_stage.h)
    if (values && c->n_runs)
        HIP_TRY(rcp::stage_d2h_i32(values, c->values.as<int32_t>(), (size_t)c->n_runs, c->device, nullptr));
    if (lengths && c->n_runs)
        HIP_TRY(rcp::stage_d2h_i32(lengths, c->lengths.as<int32_t>(), (size_t)c->n_runs, c->device, nullptr));
    if (valid && c->n_rows) HIP_TRY(rcp::stage_d2h(valid, c->valid.p, (size_t)c->n_rows, c->device, nullptr));
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_cov_free(rcp_cov* c) {
    if (c) {
        for (auto& p : c->parts) {  // each part's buffers go back to its own device's pool
            if (!p) continue;
            DeviceGuard g(p->device);
            p.reset();
        }
        DeviceGuard g(c->device);
        delete c;
    }
    return RCP_OK;
}

// =====================================================================================
// profiles of a host coverage list of Rle (the reference's $coverage object)
// =====================================================================================
namespace {

// R/profile.R slices: where -> [lo, hi) relative to the row length (see RcpPart)
bool part_slice_spec(int where, int32_t f1, int32_t f2, RcpPart* pt) {
    switch (where) {
        case RCP_WHERE_WHOLE: pt->lo_off = 0; pt->lo_end = 0; pt->hi_off = 0; pt->hi_end = 1; return true;
        case RCP_WHERE_CENTER: pt->lo_off = f1; pt->lo_end = 0; pt->hi_off = -f2; pt->hi_end = 1; return true;
        case RCP_WHERE_UPSTREAM: pt->lo_off = 0; pt->lo_end = 0; pt->hi_off = f1; pt->hi_end = 0; return true;
        case RCP_WHERE_DOWNSTREAM: pt->lo_off = -f2; pt->lo_end = 1; pt->hi_off = 0; pt->hi_end = 1; return true;
        default: return false;
    }
}

}  // namespace

namespace {

// One rcp_profile_rle call (or one row block of it) split in two: rle_prepare -- host checks and
// tasks, the runs and tables up, the run-start scan -- on one stream, and rle_finish -- the profile
// kernel and the matrix down -- on another, so that a pipeline can prepare block b + 1 while block
// b's rows come down (profile_rle_device).  The buffers are the preparing stream's; rle_prepare
// returns with its stream idle.
struct RleJob {
    explicit RleJob(hipStream_t s) : d_len(s), d_val(s), d_off(s), d_gstart(s), temp(s), d_tab(s), d_scratch(s), d_out(s) {}
    PoolBuf d_len, d_val, d_off, d_gstart, temp, d_tab, d_scratch, d_out;
    RcpRleDev P{};
    size_t lds = 0;
    bool dbl = false;
    int32_t R = 0;
    int64_t col = 0, ld = 0;
    const uint8_t* is_null = nullptr;
    std::vector<uint8_t> null_own;  // a device-resident list's NULL rows (rle_prepare with `res`)
};

// dev_rows: the row lengths and the run-length checks on the device (a row block of a big list:
// no host pass over its runs); row_base numbers the rows of the messages
// res (cov NULL): the list is a calcCoverage result still on the device (rcp_profile_cov) -- its
// runs are copied device to device, its NULL rows read from its validity; nothing crosses PCIe
int rle_prepare(const rcp_rle_desc* cov_in, const rcp_bins_desc* bins, int device, hipStream_t s, RleJob* job,
                bool dev_rows = false, int32_t row_base = 0, const rcp_cov* res = nullptr) {
    rcp_rle_desc rdesc{};
    const rcp_rle_desc* cov = cov_in;
    if (res) {
        if (res->device != device) return fail(RCP_EINVAL, "internal: coverage on device %d, not %d", res->device, device);
        rdesc.n_rows = res->n_rows;
        cov = &rdesc;
        dev_rows = true;
    }
    if (!cov || !bins) return fail(RCP_EINVAL, "NULL argument");
    const int32_t R = cov->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && !cov->run_off && !res) return fail(RCP_EINVAL, "NULL run_off");
    if (bins->n_parts < 1 || bins->n_parts > RCP_MAX_PARTS) return fail(RCP_EINVAL, "n_parts = %d", bins->n_parts);
    if (bins->stat != RCP_STAT_MEAN && bins->stat != RCP_STAT_MEDIAN) return fail(RCP_EINVAL, "stat = %d", bins->stat);
    if (bins->interp < 0 || bins->interp > 3) return fail(RCP_EINVAL, "interp = %d", bins->interp);
    if (bins->flank[0] < 0 || bins->flank[1] < 0) return fail(RCP_EINVAL, "negative flank");
    const bool dbl = cov->dvalues != nullptr;
    const int64_t n_runs = res ? res->n_runs : (R > 0 ? cov->run_off[R] : 0);
    if (!res) {
        if (R > 0 && cov->run_off[0] != 0) return fail(RCP_EINVAL, "run_off[0] != 0");
        for (int32_t r = 0; r < R; ++r)
            if (cov->run_off[r + 1] < cov->run_off[r]) return fail(RCP_EINVAL, "run_off decreases at row %d", r);
        if (n_runs > 0 && (!cov->lengths || (!cov->ivalues && !cov->dvalues)))
            return fail(RCP_EINVAL, "NULL lengths / values");
        if (cov->ivalues && cov->dvalues) return fail(RCP_EINVAL, "both integer and numeric values given");
    } else if (R > 0) {
        // the list's NULL elements: its invalid rows (calcCoverage's NULL, R/coverage.R:217-225)
        DeviceGuard gd(device);
        HIP_TRY(gd.err);
        job->null_own.resize((size_t)R);
        HIP_TRY(hipMemcpyAsync(job->null_own.data(), res->valid.p, (size_t)R, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (uint8_t& v : job->null_own) v = v ? 0 : 1;
        rdesc.is_null = job->null_own.data();
    }
    // Rle lengths are positive and every row fits int32 positions; row lengths (the slices of
    // the parts).  One pass over the runs, rows split over host threads (C4: 100 M runs).
    std::vector<int32_t> row_len(std::max(R, 1), 0);
    if (!dev_rows) {
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                                     n_runs / (1 << 20) + 1}));
        std::vector<int32_t> bad(nt, -1), big(nt, -1);
        auto work = [&](int k) {
            for (int32_t r = (int32_t)((int64_t)R * k / nt); r < (int32_t)((int64_t)R * (k + 1) / nt); ++r) {
                int64_t acc = 0;
                int32_t mn = INT32_MAX;
                for (int64_t j = cov->run_off[r]; j < cov->run_off[r + 1]; ++j) {
                    acc += cov->lengths[j];
                    mn = std::min(mn, cov->lengths[j]);
                }
                if (mn <= 0 && bad[k] < 0) bad[k] = r;
                if (acc >= (int64_t(1) << 31) && big[k] < 0) big[k] = r;
                row_len[r] = (int32_t)std::min<int64_t>(acc, INT32_MAX);
            }
        };
        if (nt == 1) {
            work(0);
        } else {
            std::vector<std::thread> th;
            for (int k = 0; k < nt; ++k) th.emplace_back(work, k);
            for (auto& t : th) t.join();
        }
        for (int k = 0; k < nt; ++k) {
            if (bad[k] >= 0) return fail(RCP_EINVAL, "row %d: an Rle run length <= 0", bad[k]);
            if (big[k] >= 0) return fail(RCP_EUNSUPPORTED, "row %d: 2^31 or more positions", big[k]);
        }
    }
    if (n_runs >= (int64_t(1) << 31)) return fail(RCP_EUNSUPPORTED, "%lld runs", (long long)n_runs);
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    HIP_TRY(g.err);
    // ---- runs to the device: lengths (+ a 0 pad for the scan), values, row offsets;
    // the scan of the lengths gives every run's start (rcp_rle.h gstart)
    PoolBuf &d_len = job->d_len, &d_val = job->d_val, &d_off = job->d_off, &d_gstart = job->d_gstart,
            &temp = job->temp;
    HIP_TRY(d_len.alloc(4 * ((size_t)n_runs + 1)));
    HIP_TRY(d_val.alloc((dbl ? 8 : 4) * std::max<size_t>((size_t)n_runs, 1)));
    HIP_TRY(d_off.alloc(8 * ((size_t)R + 1)));
    if (res) {  // device to device
        if (n_runs) {
            HIP_TRY(hipMemcpyAsync(d_len.p, res->lengths.p, 4 * (size_t)n_runs, hipMemcpyDeviceToDevice, s));
            HIP_TRY(hipMemcpyAsync(d_val.p, res->values.p, 4 * (size_t)n_runs, hipMemcpyDeviceToDevice, s));
        }
        if (R > 0) HIP_TRY(hipMemcpyAsync(d_off.p, res->run_off.p, 8 * ((size_t)R + 1), hipMemcpyDeviceToDevice, s));
    } else if (n_runs) {  // (integer runs: 16-bit offsets within blocks where they fit, rcp_stage.h)
        HIP_TRY(rcp::stage_h2d_i32(d_len.as<int32_t>(), cov->lengths, (size_t)n_runs, device, s));
        if (dbl) HIP_TRY(rcp::stage_h2d(d_val.p, cov->dvalues, 8 * (size_t)n_runs, device, s));
        else HIP_TRY(rcp::stage_h2d_i32(d_val.as<int32_t>(), cov->ivalues, (size_t)n_runs, device, s));
    }
    HIP_TRY(hipMemsetAsync(d_len.as<int32_t>() + n_runs, 0, 4, s));
    if (R > 0 && !res) HIP_TRY(rcp::stage_h2d(d_off.p, cov->run_off, 8 * ((size_t)R + 1), device, s));
    if (dev_rows && R > 0) {
        PoolBuf d_rl(s), d_bad(s);
        HIP_TRY(d_rl.alloc(4 * (size_t)R));
        HIP_TRY(d_bad.alloc(8));
        HIP_TRY(hipMemsetAsync(d_bad.p, 0x7f, 8, s));  // 0x7f7f7f7f: no such row
        HIP_TRY(rcp_rle_rowlen(R, d_off.as<int64_t>(), d_len.as<int32_t>(), d_rl.as<int32_t>(), d_bad.as<int32_t>(), s));
        int32_t h_bad[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(row_len.data(), d_rl.p, 4 * (size_t)R, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h_bad, d_bad.p, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (h_bad[0] != 0x7f7f7f7f) return fail(RCP_EINVAL, "row %d: an Rle run length <= 0", row_base + h_bad[0]);
        if (h_bad[1] != 0x7f7f7f7f)
            return fail(RCP_EUNSUPPORTED, "row %d: 2^31 or more positions", row_base + h_bad[1]);
    }
    // ---- tasks: one per (row, part), with the read path's splitVector decisions
    const bool rounding = bins->rng_kind == RCP_RNG_ROUNDING;
    RcpRleDev& P = job->P;
    std::vector<RcpRleTask> tasks;
    tasks.reserve((size_t)R * bins->n_parts);
    std::vector<int32_t> lay_cnt, nb_pos;
    std::map<std::pair<int, int>, int32_t> layout_cache, nb_cache;
    int64_t col = 0;
    int32_t max_interp_len = 0, max_interp_bins = 0, n_scratch = 0;
    for (int p = 0; p < bins->n_parts; ++p) {
        RcpPart pt{};
        if (!part_slice_spec(bins->where ? bins->where[p] : RCP_WHERE_WHOLE, bins->flank[0], bins->flank[1], &pt))
            return fail(RCP_EINVAL, "where[%d] = %d", p, bins->where[p]);
        const int nb = bins->n_bins[p];
        if (nb < 0) return fail(RCP_EINVAL, "n_bins[%d] < 0", p);
        const bool per_base = nb == 0;
        const int32_t ncol = per_base ? (bins->per_base_width ? bins->per_base_width[p] : 0) : nb;
        if (ncol <= 0) return fail(RCP_EINVAL, "part %d has no columns", p);
        P.part_col0[p] = (int32_t)col;
        P.part_cols[p] = ncol;
        col += ncol;
        for (int32_t r = 0; r < R; ++r) {
            RcpRleTask t{};
            t.row = r;
            t.part = p;
            t.lay = t.nbpos = t.scratch = -1;
            if (cov->is_null && cov->is_null[r]) {
                t.mode = RCP_RLE_ZERO;
                tasks.push_back(t);
                continue;
            }
            int32_t head, L;
            rcp_part_slice(pt, row_len[r], &head, &L);
            if (L < 0 || head < 0 || head + L > row_len[r])
                return fail(RCP_EUNSUPPORTED, "row %d: part %d slice out of its %d-long coverage", r, p, row_len[r]);
            t.head = head;
            t.L = L;
            if (per_base) {
                if (L != ncol)
                    return fail(RCP_EUNSUPPORTED, "a per-base part met a row whose slice width differs from the column count");
                t.mode = RCP_RLE_BASE;
            } else if (L < nb) {
                int mode = bins->interp;
                if (mode == RCP_INTERP_AUTO)
                    mode = ((double)(nb - L) / nb < 0.2) ? RCP_INTERP_NEIGHBORHOOD : RCP_INTERP_SPLINE;
                if (mode == RCP_INTERP_NEIGHBORHOOD) {
                    const auto key = std::make_pair(nb, L);
                    auto it = nb_cache.find(key);
                    if (it == nb_cache.end()) {
                        std::vector<int32_t> pos;
                        if (!rcp::neighborhood_positions(nb, L, rounding, &pos))
                            return fail(RCP_ESEMANTIC,
                                        "splitVector neighborhood interpolation of %d values into %d bins: R raises an error",
                                        L, nb);
                        t.nbpos = (int32_t)nb_pos.size();
                        nb_pos.insert(nb_pos.end(), pos.begin(), pos.end());
                        nb_cache[key] = t.nbpos;
                    } else {
                        t.nbpos = it->second;
                    }
                } else if (mode == RCP_INTERP_SPLINE && L < 1) {
                    return fail(RCP_ESEMANTIC, "spline() of zero points: R raises an error");
                } else if (mode == RCP_INTERP_LINEAR && L < 1) {
                    return fail(RCP_EUNSUPPORTED, "empty slice with the 'linear' interpolation");
                }
                t.mode = RCP_RLE_INTERP + mode;
                t.scratch = n_scratch++;
                max_interp_len = std::max(max_interp_len, L);
                max_interp_bins = std::max(max_interp_bins, nb);
            } else {
                t.mode = RCP_RLE_BINNED;
                t.bs = L / nb;
                const int32_t dif = L - t.bs * nb;
                if (dif) {
                    const auto key = std::make_pair(nb, dif);
                    auto it = layout_cache.find(key);
                    if (it == layout_cache.end()) {
                        const std::vector<int32_t> cnt = rcp::bin_layout_counts(nb, dif, rounding);
                        t.lay = (int32_t)lay_cnt.size();
                        lay_cnt.insert(lay_cnt.end(), cnt.begin(), cnt.end());
                        layout_cache[key] = t.lay;
                    } else {
                        t.lay = it->second;
                    }
                }
            }
            tasks.push_back(t);
        }
    }
    if (max_interp_len > kChunkMax)
        return fail(RCP_EUNSUPPORTED, "interpolated slice of %d positions exceeds %d", max_interp_len, kChunkMax);
    // fmm pivots (as rcp_plan_create)
    std::vector<double> spl_tb(2 * ((size_t)std::max(max_interp_len, 1) + 1), 0.0);
    {
        double bp = -1.0;
        spl_tb[1] = bp;
        for (size_t i = 1; 2 * i + 1 < spl_tb.size(); ++i) {
            const double t = 1.0 / bp;
            bp = 4.0 - t;
            spl_tb[2 * i] = t;
            spl_tb[2 * i + 1] = bp;
        }
    }
    // interpolation working set: x (L+1) | y (n+1) | b, c, d (3 (L+1)) | n ints
    // (the neighborhood fill's n pre-fill values reuse b.., as in rcp_plan_create)
    const int64_t stride = ((int64_t)max_interp_len + 1) +
                           std::max<int64_t>(max_interp_bins, 3 * ((int64_t)max_interp_len + 1)) + 8;
    const size_t lds = n_scratch ? 8 * (size_t)stride : 0;
    P.interp_lds = lds <= 160 * 1024 ? 1 : 0;
    P.interp_stride = stride;
    std::vector<RcpRleTask> itasks;
    // run starts: from the lengths inside the tile kernel when every part's slice starts at the
    // row's first position and no row is interpolated or a median (each row is streamed from
    // its first run); else one device scan of the lengths (the starts the searches need)
    bool from_lengths = bins->stat == RCP_STAT_MEAN;
    for (int p = 0; p < bins->n_parts; ++p) {
        RcpPart pt{};
        part_slice_spec(bins->where ? bins->where[p] : RCP_WHERE_WHOLE, bins->flank[0], bins->flank[1], &pt);
        if (pt.lo_end != 0 || pt.lo_off != 0) from_lengths = false;
    }
    for (int p = 0; p < bins->n_parts; ++p) P.part_dense[p] = dbl ? 0 : 1;
    for (const RcpRleTask& t : tasks) {
        if (t.mode >= RCP_RLE_INTERP) itasks.push_back(t);
        // dense windows: integer means of uniform 1-, 2- or 4-position bins, or per-base values
        const bool dense_ok = t.mode == RCP_RLE_ZERO || t.mode >= RCP_RLE_INTERP || t.mode == RCP_RLE_BASE ||
                              (t.mode == RCP_RLE_BINNED && bins->stat == RCP_STAT_MEAN && t.lay < 0 &&
                               (t.bs == 1 || t.bs == 2 || t.bs == 4));
        if (!dense_ok) P.part_dense[t.part] = 0;
    }
    std::vector<char> blob;
    const size_t o_tasks = put(blob, tasks);
    const size_t o_itasks = put(blob, itasks);
    if (!itasks.empty()) from_lengths = false;
    if (!from_lengths) {
        size_t tb = 0;
        HIP_TRY(d_gstart.alloc(8 * ((size_t)n_runs + 1)));
        HIP_TRY(rcp_rle_scan(d_len.as<int32_t>(), n_runs, d_gstart.as<int64_t>(), nullptr, &tb, s));
        HIP_TRY(temp.alloc(std::max<size_t>(tb, 1)));
        HIP_TRY(rcp_rle_scan(d_len.as<int32_t>(), n_runs, d_gstart.as<int64_t>(), temp.p, &tb, s));
    }
    const size_t o_lay = put(blob, lay_cnt);
    const size_t o_nb = put(blob, nb_pos);
    const size_t o_spl = put(blob, spl_tb);
    PoolBuf &d_tab = job->d_tab, &d_scratch = job->d_scratch, &d_out = job->d_out;
    HIP_TRY(d_tab.alloc(blob.size()));
    HIP_TRY(rcp::stage_h2d(d_tab.p, blob.data(), blob.size(), device, s));
    if (n_scratch && !P.interp_lds) HIP_TRY(d_scratch.alloc(8 * (size_t)stride * n_scratch));
    const int64_t ld = ((int64_t)R + 15) & ~int64_t(15);
    HIP_TRY(d_out.alloc(8 * std::max<size_t>((size_t)ld * (size_t)col, 1)));
    char* base = d_tab.as<char>();
    P.run_off = d_off.as<int64_t>();
    P.gstart = from_lengths ? nullptr : d_gstart.as<int64_t>();
    P.lengths = d_len.as<int32_t>();
    P.ivals = dbl ? nullptr : d_val.as<int32_t>();
    P.dvals = dbl ? d_val.as<double>() : nullptr;
    P.tasks = reinterpret_cast<const RcpRleTask*>(base + o_tasks);
    P.n_rows = R;
    P.n_parts = bins->n_parts;
    P.itasks = reinterpret_cast<const RcpRleTask*>(base + o_itasks);
    P.n_itasks = (int64_t)itasks.size();
    P.lay_cnt = reinterpret_cast<const int32_t*>(base + o_lay);
    P.nb_pos = reinterpret_cast<const int32_t*>(base + o_nb);
    P.spl_tb = reinterpret_cast<const double*>(base + o_spl);
    P.out = d_out.as<double>();
    P.ld = ld;
    P.stat = bins->stat;
    P.scale = bins->scale;
    P.scratch = d_scratch.as<double>();
    job->lds = P.interp_lds ? lds : 0;
    job->dbl = dbl;
    job->R = R;
    job->col = col;
    job->ld = ld;
    job->is_null = cov->is_null;
    HIP_TRY(hipStreamSynchronize(s));
    return RCP_OK;
}

int rle_finish_run(RleJob* job, int device, double* out, int64_t out_ld, uint8_t* row_valid, hipStream_t s) {
    DeviceGuard g(device);
    HIP_TRY(g.err);
    HIP_TRY(rcp_rle_profile_launch(&job->P, job->dbl ? 1 : 0, job->lds, s));
    const size_t R = (size_t)job->R, C = (size_t)job->col;
    const RcpRleDev& P = job->P;
    // integer Rle, one part of mean bins: the matrix as numerators (download_matrix)
    if (out && R && C && !job->dbl && P.n_parts == 1 && P.stat == 0 && (size_t)P.n_itasks <= R / 8 && P.scale > 0.0 &&
        std::isfinite(P.scale) && C <= 65535u * 8u && 8 * R * C >= (size_t(4) << 20)) {
        const int e = download_packed(job->d_out.as<double>(), (size_t)job->ld, R, C, P.scale, out, (size_t)out_ld,
                                      device, s, [&](uint32_t* q, uint32_t* div, uint32_t* bad) {
                                          return rcp_rle_pack(&P, (int64_t)C, q, div, bad, s);
                                      });
        if (e) return e;
    } else if (out && R && C) {
        HIP_TRY(rcp::stage_d2h_2d(out, 8 * (size_t)out_ld, job->d_out.p, 8 * (size_t)job->ld, 8 * R, C, device, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (row_valid)
        for (int32_t r = 0; r < job->R; ++r) row_valid[r] = (job->is_null && job->is_null[r]) ? 0 : 1;
    return RCP_OK;
}

// The profile of a prepared job and its rows down; on every exit the stream has drained, so the
// caller may hand the job's pool buffers back (they are recorded idle on the preparer's stream,
// while the kernel ran on `s`)
int rle_finish(RleJob* job, int device, double* out, int64_t out_ld, uint8_t* row_valid, hipStream_t s) {
    const int rc = rle_finish_run(job, device, out, out_ld, row_valid, s);
    if (rc != RCP_OK) {
        DeviceGuard g(device);
        (void)hipStreamSynchronize(s);
        (void)hipGetLastError();
    }
    return rc;
}

}  // namespace

int rcpi::profile_rle_impl(const rcp_rle_desc* cov, const rcp_bins_desc* bins, int device, double* out,
                           int64_t out_ld, uint8_t* row_valid, hipStream_t s) {
    RleJob job(s);
    const int rc = rle_prepare(cov, bins, device, s, &job);
    if (rc) return rc;
    return rle_finish(&job, device, out, out_ld, row_valid, s);
}

namespace {

// rcp_profile_rle of rows [0, cov->n_rows) on one device, into a matrix of column stride out_ld:
// a big list goes in row blocks through three host threads -- one prepares each block (host
// checks and tasks, its runs up through the upload staging buffers), two finish them in turn
// (profile kernel, the block's rows of the matrix down through the download staging buffers) --
// so that block b + 1's runs go up while block b's rows come down (PCIe is full duplex; the
// staging buffers are per direction, rcp_stage.cpp): C4's 0.8 GB of runs up and 1.6 GB of
// matrix down overlap.  At most three blocks are on the device.
int profile_rle_device(const rcp_rle_desc* cov, const rcp_bins_desc* bins, int device, double* out, int64_t out_ld,
                       uint8_t* row_valid) {
    const int32_t R = cov->n_rows;
    const int64_t n_runs = R > 0 ? cov->run_off[R] : 0;
    int nb = 1;  // row blocks
    if (n_runs >= (int64_t(1) << 23) && R >= 4096) nb = 8;
    else if (n_runs >= (int64_t(1) << 21) && R >= 1024) nb = 4;
    // (one block, or no such device: the single call validates the lists before any device work)
    if (nb == 1 || check_device(device) != RCP_OK)
        return profile_rle_impl(cov, bins, device, out, out_ld, row_valid, nullptr);
    std::vector<double> cum((size_t)R + 1, 0.0);
    for (int32_t r = 0; r < R; ++r) cum[r + 1] = cum[r] + 64.0 + (double)(cov->run_off[r + 1] - cov->run_off[r]);
    const std::vector<int32_t> split = balanced_split(cum, nb);
    struct Block {
        int b;
        std::unique_ptr<RleJob> job;
    };
    std::deque<Block> ready;
    int in_flight = 0;  // being prepared or prepared, not yet finished
    int next_b = 0, preparers_left = 2;
    bool abort = false;
    std::mutex mu;
    std::condition_variable cv;
    const bool tr = rcp::trace_on();
    const double t0 = tr ? rcp::trace_ms() : 0.0;
    // the preparers' streams outlive every job (their buffers are freed on them)
    DeviceGuard g(device);
    HIP_TRY(g.err);
    hipStream_t sp[2] = {nullptr, nullptr};
    struct Streams {
        hipStream_t* v;
        ~Streams() {
            for (int i = 0; i < 2; ++i)
                if (v[i]) (void)hipStreamDestroy(v[i]);
        }
    } spguard{sp};
    for (int i = 0; i < 2; ++i) HIP_TRY(hipStreamCreateWithFlags(&sp[i], hipStreamNonBlocking));
    // two preparers (the host checks and tasks of one block beside the other's uploads) and two
    // finishers (one block's kernel and plan beside the other's download); at most four blocks
    const int rc = run_per_device(4, [&](int role) -> int {
        DeviceGuard gt(device);
        HIP_TRY(gt.err);
        hipStream_t s = role < 2 ? sp[role] : nullptr;
        std::unique_ptr<std::remove_pointer<hipStream_t>::type, hipError_t (*)(hipStream_t)> sguard(nullptr,
                                                                                                     hipStreamDestroy);
        if (role >= 2) {
            HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            sguard.reset(s);
        }
        if (role < 2) {  // preparers
            auto done = [&] {
                {
                    std::lock_guard<std::mutex> lock(mu);
                    --preparers_left;
                }
                cv.notify_all();
            };
            for (;;) {
                int b;
                {
                    std::unique_lock<std::mutex> lock(mu);
                    cv.wait(lock, [&] { return abort || in_flight < 4 || next_b >= nb; });
                    if (abort) return (int)RCP_OK;
                    if (next_b >= nb) break;
                    b = next_b++;
                    ++in_flight;
                }
                const int32_t r0 = split[b], r1 = split[b + 1];
                if (r1 <= r0) {
                    std::lock_guard<std::mutex> lock(mu);
                    --in_flight;
                    continue;
                }
                // the block as an Rle list of its own: run offsets from 0, arrays from its first run
                const int64_t base = cov->run_off[r0];
                std::vector<int64_t> off((size_t)(r1 - r0) + 1);
                for (int32_t r = r0; r <= r1; ++r) off[r - r0] = cov->run_off[r] - base;
                rcp_rle_desc sub = *cov;
                sub.n_rows = r1 - r0;
                sub.run_off = off.data();
                sub.lengths = cov->lengths ? cov->lengths + base : nullptr;
                sub.ivalues = cov->ivalues ? cov->ivalues + base : nullptr;
                sub.dvalues = cov->dvalues ? cov->dvalues + base : nullptr;
                sub.is_null = cov->is_null ? cov->is_null + r0 : nullptr;
                const double tb = tr ? rcp::trace_ms() : 0.0;
                auto job = std::make_unique<RleJob>(s);
                const int e = rle_prepare(&sub, bins, device, s, job.get(), true, r0);
                if (tr)
                    fprintf(stderr, "[rle] block %d rows [%d, %d): prepared %.2f ms (at %.2f)\n", b, r0, r1,
                            rcp::trace_ms() - tb, tb - t0);
                {
                    std::lock_guard<std::mutex> lock(mu);
                    if (e) {
                        abort = true;
                    } else {
                        ready.push_back(Block{b, std::move(job)});
                    }
                }
                cv.notify_all();
                if (e) {
                    done();
                    return e;
                }
            }
            done();
            return (int)RCP_OK;
        }
        for (;;) {  // finishers
            Block blk;
            {
                std::unique_lock<std::mutex> lock(mu);
                cv.wait(lock, [&] { return abort || !ready.empty() || preparers_left == 0; });
                if (abort || ready.empty()) return (int)RCP_OK;
                blk = std::move(ready.front());
                ready.pop_front();
            }
            const int32_t r0 = split[blk.b];
            const double tb = tr ? rcp::trace_ms() : 0.0;
            const int e = rle_finish(blk.job.get(), device, out ? out + r0 : nullptr, out_ld,
                                     row_valid ? row_valid + r0 : nullptr, s);
            if (tr)
                fprintf(stderr, "[rle] block %d: profiled + down %.2f ms (at %.2f)\n", blk.b, rcp::trace_ms() - tb,
                        tb - t0);
            blk.job.reset();  // (its buffers back to the cache: this stream is idle)
            {
                std::lock_guard<std::mutex> lock(mu);
                --in_flight;
                if (e) abort = true;
            }
            cv.notify_all();
            if (e) return e;
        }
    });
    ready.clear();  // (left by a failure: freed while the preparer's stream exists)
    return rc;
}

}  // namespace

extern "C" int rcp_profile_rle(const rcp_rle_desc* cov, const rcp_bins_desc* bins, int device, double* out,
                               uint8_t* row_valid) {
    RCP_TRY
    if (!cov || !bins) return fail(RCP_EINVAL, "NULL argument");
    const int32_t R = cov->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && !cov->run_off) return fail(RCP_EINVAL, "NULL run_off");
    if (R > 0 && cov->run_off[0] != 0) return fail(RCP_EINVAL, "run_off[0] != 0");
    for (int32_t r = 0; r < R; ++r)
        if (cov->run_off[r + 1] < cov->run_off[r]) return fail(RCP_EINVAL, "run_off decreases at row %d", r);
    return profile_rle_device(cov, bins, device, out, R, row_valid);
    RCP_CATCH
}

extern "C" int rcp_profile_rle_multi(const rcp_rle_desc* cov, const rcp_bins_desc* bins, const int32_t* device_ids,
                                     int32_t n_devices, double* out, uint8_t* row_valid) {
    RCP_TRY
    if (!cov || !bins || !device_ids) return fail(RCP_EINVAL, "NULL argument");
    if (n_devices < 1 || n_devices > 64) return fail(RCP_EINVAL, "n_devices = %d", n_devices);
    for (int i = 0; i < n_devices; ++i) {
        const int rc = check_device(device_ids[i]);
        if (rc) return rc;
    }
    const int32_t R = cov->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && !cov->run_off) return fail(RCP_EINVAL, "NULL run_off");
    if (R > 0 && cov->run_off[0] != 0) return fail(RCP_EINVAL, "run_off[0] != 0");
    for (int32_t r = 0; r < R; ++r)
        if (cov->run_off[r + 1] < cov->run_off[r]) return fail(RCP_EINVAL, "run_off decreases at row %d", r);
    if (n_devices == 1) return profile_rle_device(cov, bins, device_ids[0], out, R, row_valid);
    // contiguous row blocks balanced by the runs each row streams (12 bytes each up, read once)
    // plus its output columns (the same for every row: a constant per row)
    std::vector<double> cum((size_t)R + 1, 0.0);
    for (int32_t r = 0; r < R; ++r) cum[r + 1] = cum[r] + 64.0 + (double)(cov->run_off[r + 1] - cov->run_off[r]);
    const std::vector<int32_t> split = balanced_split(cum, n_devices);
    return run_per_device(n_devices, [&](int i) {
        const int32_t r0 = split[i], r1 = split[i + 1];
        if (r1 <= r0) return (int)RCP_OK;
        // the block as an Rle list of its own: run offsets from 0, arrays from its first run
        const int64_t base = cov->run_off[r0];
        std::vector<int64_t> off((size_t)(r1 - r0) + 1);
        for (int32_t r = r0; r <= r1; ++r) off[r - r0] = cov->run_off[r] - base;
        rcp_rle_desc sub = *cov;
        sub.n_rows = r1 - r0;
        sub.run_off = off.data();
        sub.lengths = cov->lengths ? cov->lengths + base : nullptr;
        sub.ivalues = cov->ivalues ? cov->ivalues + base : nullptr;
        sub.dvalues = cov->dvalues ? cov->dvalues + base : nullptr;
        sub.is_null = cov->is_null ? cov->is_null + r0 : nullptr;
        return profile_rle_device(&sub, bins, device_ids[i], out ? out + r0 : nullptr, R,
                                  row_valid ? row_valid + r0 : nullptr);
    });
    RCP_CATCH
}

extern "C" int rcp_profile_cov(const rcp_cov* c, const rcp_bins_desc* bins, double* out, uint8_t* row_valid) {
    RCP_TRY
    if (!c || !bins) return fail(RCP_EINVAL, "NULL argument");
    if (bins->n_parts < 1 || bins->n_parts > RCP_MAX_PARTS) return fail(RCP_EINVAL, "n_parts = %d", bins->n_parts);
    const int32_t R = c->n_rows;
    auto one = [&](const rcp_cov* part, double* o, int64_t ld, uint8_t* v) -> int {
        RleJob job(nullptr);
        const int rc = rle_prepare(nullptr, bins, part->device, nullptr, &job, true, 0, part);
        if (rc) return rc;
        return rle_finish(&job, part->device, o, ld, v, nullptr);
    };
    if (c->parts.empty()) return one(c, out, R, row_valid);
    // several devices' row blocks (rcp_shards_coverage): each block profiled on its own device, its
    // rows into the caller's matrix -- in place when the blocks are the caller's row ranges, else
    // through a host matrix of the block scattered to the caller's rows (the shards' order)
    int64_t C = 0;
    for (int p = 0; p < bins->n_parts; ++p)
        C += bins->n_bins[p] ? bins->n_bins[p] : (bins->per_base_width ? bins->per_base_width[p] : 0);
    const int np = (int)c->parts.size();
    return run_per_device(np, [&](int b) -> int {
        const rcp_cov* p = c->parts[b].get();
        const int32_t r0 = c->split[b], n = p->n_rows;
        if (n == 0) return (int)RCP_OK;
        if (c->order.empty()) return one(p, out ? out + r0 : nullptr, R, row_valid ? row_valid + r0 : nullptr);
        std::vector<double> tmp(out ? (size_t)n * (size_t)C : 0);
        std::vector<uint8_t> v((size_t)n);
        const int rc = one(p, out ? tmp.data() : nullptr, n, v.data());
        if (rc) return rc;
        for (int32_t i = 0; i < n; ++i) {
            const int32_t r = c->order[(size_t)r0 + i];
            if (row_valid) row_valid[r] = v[i];
            if (out)
                for (int64_t k = 0; k < C; ++k) out[(size_t)k * R + r] = tmp[(size_t)k * n + i];
        }
        return (int)RCP_OK;
    });
    RCP_CATCH
}

// =====================================================================================
// R RNG for the preprocessing steps (downsample / sampleto, R/ranges.R:32-62)
// =====================================================================================
struct rcp_rng {
    rcp::RRng rng;
    bool rounding;
    rcp_rng(uint32_t seed, bool r) : rng(seed), rounding(r) {}
};

extern "C" int rcp_rng_create(uint32_t seed, int kind, rcp_rng** out) {
    RCP_TRY
    if (!out) return fail(RCP_EINVAL, "NULL argument");
    if (kind != RCP_RNG_REJECTION && kind != RCP_RNG_ROUNDING) return fail(RCP_EINVAL, "rng kind %d", kind);
    *out = new rcp_rng(seed, kind == RCP_RNG_ROUNDING);
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_rng_unif(rcp_rng* g, int64_t k, double* out) {
    RCP_TRY
    if (!g || (k > 0 && !out)) return fail(RCP_EINVAL, "NULL argument");
    for (int64_t i = 0; i < k; ++i) out[i] = g->rng.unif_rand();
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_rng_sample_sorted(rcp_rng* g, int64_t n, int64_t k, int64_t* out) {
    RCP_TRY
    if (!g || (k > 0 && !out)) return fail(RCP_EINVAL, "NULL argument");
    std::vector<int64_t> v;
    if (!g->rng.sample_sorted(n, k, g->rounding, &v))
        return fail(RCP_ESEMANTIC, "cannot take a sample larger than the population when 'replace = FALSE'");
    std::copy(v.begin(), v.end(), out);
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_rng_free(rcp_rng* g) {
    RCP_TRY
    delete g;
    return RCP_OK;
    RCP_CATCH
}
