// rcp_shard.cpp -- one sample's reads split over several GPUs for one region table (the C ABI's
// rcp_shards_*; include/recoup_amd.h).
//
// The reference's only parallelism is cmclapply over the regions of calcCoverage
// (R/coverage.R:147-154) and over the rows of binCoverageMatrix (R/profile.R:198-199;
// R/util.R:364-382).  Here the regions are cut into one contiguous row block per GPU, balanced by
// the candidate reads the GPUs count for every row, and each GPU holds only the reads its block's
// regions can overlap:
//   A  the reads are uploaded in n_devices slices, one per GPU (every PCIe link at once); each
//      GPU sorts its slice into a search index (rcp_readset, no bucket directory);
//   B  each GPU counts, per region range and strand stream, the candidate reads of its slice
//      (rcp_seg_bounds_kernel); the host sums them per row and cuts the blocks;
//   C  each GPU gathers, for every block, the reads of its slice inside the block's candidate
//      ranges (rcp_gather_kernel) and copies them device to device (xGMI) into that block's GPU;
//   D  each GPU builds the readset of its block from what it received (the layout the row table
//      searches: strand-merged for ignore.strand = TRUE, strand-split for FALSE).
// A read several blocks overlap goes to each of them; nothing else is duplicated.  A row sees
// exactly the reads findOverlaps hits on one device, so every result is bit-identical to a single
// device (the NULL rules read only the hits: R/coverage.R:189-225).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "rcp_internal.h"
#include "rcp_stage.h"

extern "C" {
hipError_t rcp_launch_seg_bounds(int64_t n_seg, const int32_t* chrom, const int32_t* start, const int32_t* end,
                                 const int8_t* strand, int merged, int32_t n_chrom, const int64_t* stream_off,
                                 const int32_t* pmax, const int2* se, uint2* out, hipStream_t stream);
hipError_t rcp_launch_gather(int64_t n_out, int64_t n_ranges, const int64_t* out_off, const uint32_t* lo,
                             const int32_t* sid, const int2* se, int32_t* chrom_out, int32_t* start_out,
                             int32_t* end_out, int8_t* strand_out, hipStream_t stream);
}

using namespace rcpi;

struct rcp_shards {
    std::vector<int32_t> devices;
    std::vector<rcp_readset*> rs;  // one per device (the block's reads)
    std::vector<int32_t> split;    // row blocks [split[b], split[b + 1]) of the table in (chrom, start) order
    std::vector<int32_t> order;    // the caller's row at each position of that order (empty: the caller's
                                   // table is in that order already)
    // the row table (a copy: the caller's arrays may go away)
    int32_t n_rows = 0;
    std::vector<int64_t> seg_off;
    std::vector<int32_t> chrom, start, end;
    std::vector<int8_t> strand, group;
    uint8_t is_list[4] = {0, 0, 0, 0};
    bool has_group = false, has_list = false;
    int32_t ignore_strand = 1;

    rcp_rows_desc rows() const {
        rcp_rows_desc d{};
        d.n_rows = n_rows;
        d.seg_off = seg_off.data();
        d.seg_chrom = chrom.data();
        d.seg_start = start.data();
        d.seg_end = end.data();
        d.seg_strand = strand.data();
        d.seg_group = has_group ? group.data() : nullptr;
        d.group_is_list = has_list ? is_list : nullptr;
        d.ignore_strand = ignore_strand;
        return d;
    }
    rcp_rows_desc block(int b) const {  // seg_off indexes the shared segment arrays directly
        rcp_rows_desc d = rows();
        d.n_rows = split[b + 1] - split[b];
        d.seg_off = seg_off.data() + split[b];
        return d;
    }
    ~rcp_shards() {
        for (rcp_readset* r : rs) rcp_readset_destroy(r);
    }
};

namespace rcpi {

int seg_bounds(const rcp_readset* rs, const rcp_rows_desc* rows, std::vector<uint2>* out) {
    const int64_t n_seg = rows->n_rows > 0 ? rows->seg_off[rows->n_rows] : 0;
    out->assign(3 * (size_t)std::max<int64_t>(n_seg, 0), make_uint2(0u, 0u));
    if (n_seg <= 0) return RCP_OK;
    const bool merged = rows->ignore_strand != 0;
    const ReadLayout& L = merged ? rs->merged : rs->stranded;
    if (merged ? !rs->has_merged : !rs->stranded_ready)
        return fail(RCP_EINVAL, "internal: the readset lacks the %s layout", merged ? "merged" : "strand-split");
    if (rs->n == 0) return RCP_OK;
    DeviceGuard g(rs->device);
    HIP_TRY(g.err);
    hipStream_t s = nullptr;
    PoolBuf d_seg(s), d_out(s);
    const size_t n = (size_t)n_seg;
    HIP_TRY(d_seg.alloc(13 * n));
    int32_t* dc = d_seg.as<int32_t>();
    int8_t* dst = reinterpret_cast<int8_t*>(dc + 3 * n);
    HIP_TRY(hipMemcpyAsync(dc, rows->seg_chrom, 4 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dc + n, rows->seg_start, 4 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dc + 2 * n, rows->seg_end, 4 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dst, rows->seg_strand, n, hipMemcpyHostToDevice, s));
    HIP_TRY(d_out.alloc(8 * 3 * n));
    HIP_TRY(rcp_launch_seg_bounds(n_seg, dc, dc + n, dc + 2 * n, dst, merged ? 1 : 0, rs->n_chrom,
                                  L.stream_off.as<int64_t>(), L.pmax.as<int32_t>(), L.se.as<int2>(),
                                  d_out.as<uint2>(), s));
    HIP_TRY(hipMemcpyAsync(out->data(), d_out.p, 8 * 3 * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return RCP_OK;
}

int cov_copy_parts(const rcp_cov* c, int64_t* run_off, int32_t* values, int32_t* lengths, uint8_t* valid) {
    const int np = (int)c->parts.size();
    if (!c->order.empty()) {
        // the parts hold rows in (chrom, start) order: each part's runs come into host arrays of its
        // own, then every row's runs go to the caller's row (offsets from the caller-order counts)
        std::vector<std::vector<int64_t>> off(np);
        std::vector<std::vector<uint8_t>> val(np);
        int rc = run_per_device(np, [&](int b) {
            const rcp_cov* p = c->parts[b].get();
            off[b].assign((size_t)p->n_rows + 1, 0);
            val[b].assign((size_t)std::max(p->n_rows, 1), 0);
            return rcp_cov_copy(p, off[b].data(), nullptr, nullptr, val[b].data());
        });
        if (rc) return rc;
        std::vector<int64_t> at((size_t)c->n_rows + 1, 0);  // caller-order run offsets
        for (int b = 0; b < np; ++b)
            for (int32_t i = 0; i < c->parts[b]->n_rows; ++i) {
                const int32_t r = c->order[(size_t)c->split[b] + i];
                at[(size_t)r + 1] = off[b][i + 1] - off[b][i];
                if (valid) valid[r] = val[b][i];
            }
        for (int32_t r = 0; r < c->n_rows; ++r) at[(size_t)r + 1] += at[r];
        if (run_off) std::copy(at.begin(), at.end(), run_off);
        if (!values && !lengths) return RCP_OK;
        return run_per_device(np, [&](int b) {
            const rcp_cov* p = c->parts[b].get();
            std::vector<int32_t> v((size_t)std::max<int64_t>(p->n_runs, 1)), l(v.size());
            int e = rcp_cov_copy(p, nullptr, values ? v.data() : nullptr, lengths ? l.data() : nullptr, nullptr);
            if (e) return e;
            for (int32_t i = 0; i < p->n_rows; ++i) {
                const int64_t a = off[b][i], k = off[b][i + 1] - a;
                const size_t to = (size_t)at[c->order[(size_t)c->split[b] + i]];
                if (values) std::memcpy(values + to, v.data() + a, 4 * (size_t)k);
                if (lengths) std::memcpy(lengths + to, l.data() + a, 4 * (size_t)k);
            }
            return (int)RCP_OK;
        });
    }
    // each part's runs land at its place in the caller's arrays (the parts' rows and runs are
    // consecutive blocks of the whole list), one host thread per part; its run offsets are
    // shifted by the runs of the parts before it
    std::vector<int64_t> base(np + 1, 0);
    for (int b = 0; b < np; ++b) base[b + 1] = base[b] + c->parts[b]->n_runs;
    const int rc = run_per_device(np, [&](int b) {
        const rcp_cov* p = c->parts[b].get();
        const int32_t r0 = c->split[b];
        std::vector<int64_t> off((size_t)p->n_rows + 1, 0);
        int e = rcp_cov_copy(p, run_off ? off.data() : nullptr, values ? values + base[b] : nullptr,
                             lengths ? lengths + base[b] : nullptr, valid ? valid + r0 : nullptr);
        if (e) return e;
        if (run_off)
            for (int32_t r = 0; r < p->n_rows; ++r) run_off[r0 + r] = base[b] + off[r];
        return (int)RCP_OK;
    });
    if (rc) return rc;
    if (run_off) run_off[c->n_rows] = base[np];
    return RCP_OK;
}

}  // namespace rcpi

namespace {

// The runs (value, length) of an Rle restricted to elements [a, b)
void slice_runs(const int32_t* val, const int64_t* len, int32_t n_runs, int64_t a, int64_t b,
                std::vector<int32_t>* v, std::vector<int64_t>* l) {
    v->clear();
    l->clear();
    int64_t pos = 0;
    for (int32_t k = 0; k < n_runs && pos < b; ++k) {
        const int64_t lo = std::max(pos, a), hi = std::min(pos + len[k], b);
        if (hi > lo) {
            v->push_back(val[k]);
            l->push_back(hi - lo);
        }
        pos += len[k];
    }
}

}  // namespace

void rcpi::slice_reads(const rcp_reads_desc* src, int64_t a, int64_t b, ReadSlice* out) {
    rcp_reads_desc& d = out->d;
    d = *src;
    d.n = b - a;
    // (per-read arrays: host or device pointers; the runs are host arrays in both modes)
    if (src->chrom) {
        d.chrom = src->chrom + a;
    } else if (d.n > 0) {
        slice_runs(src->chrom_run_value, src->chrom_run_length, src->n_chrom_runs, a, b, &out->cv, &out->cl);
        d.n_chrom_runs = (int32_t)out->cv.size();
        d.chrom_run_value = out->cv.data();
        d.chrom_run_length = out->cl.data();
    }
    if (src->end) {
        d.end = src->end + a;
    } else if (d.n > 0) {
        slice_runs(src->width_run_value, src->width_run_length, src->n_width_runs, a, b, &out->wv, &out->wl);
        d.n_width_runs = (int32_t)out->wv.size();
        d.width_run_value = out->wv.data();
        d.width_run_length = out->wl.data();
    }
    if (d.start) d.start = src->start + a;
    if (d.strand) d.strand = src->strand + a;
}

namespace {

// Enable direct device-to-device copies between every pair of the listed GPUs (xGMI), once per
// pair; where that is refused the copies below still run (staged by the runtime).
void enable_peers(const std::vector<int32_t>& devices) {
    static std::mutex mu;
    static std::vector<std::pair<int, int>> done;
    std::lock_guard<std::mutex> lock(mu);
    for (int32_t a : devices)
        for (int32_t b : devices) {
            if (a == b || std::find(done.begin(), done.end(), std::make_pair(a, b)) != done.end()) continue;
            done.emplace_back(a, b);
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
            DeviceGuard g(a);
            (void)hipDeviceEnablePeerAccess(b, 0);
            (void)hipGetLastError();  // "already enabled" is not an error here
        }
}

struct Range {
    int32_t sid;
    uint32_t lo, hi;
};

}  // namespace

extern "C" int rcp_shards_create(const rcp_reads_desc* reads, const rcp_rows_desc* rows, const int32_t* device_ids,
                                 int32_t n_devices, rcp_shards** out) {
    RCP_TRY
    if (!reads || !rows || !device_ids || !out) return fail(RCP_EINVAL, "NULL argument");
    *out = nullptr;
    if (n_devices < 1 || n_devices > 64) return fail(RCP_EINVAL, "n_devices = %d", n_devices);
    for (int i = 0; i < n_devices; ++i) {
        const int rc = check_device(device_ids[i]);
        if (rc) return rc;
    }
    const int32_t R = rows->n_rows;
    if (R < 0) return fail(RCP_EINVAL, "n_rows < 0");
    if (R > 0 && (!rows->seg_off || !rows->seg_chrom || !rows->seg_start || !rows->seg_end || !rows->seg_strand))
        return fail(RCP_EINVAL, "NULL row array");
    if (R > 0 && rows->seg_off[0] != 0) return fail(RCP_EINVAL, "seg_off[0] != 0");
    for (int32_t r = 0; r < R; ++r)
        if (rows->seg_off[r + 1] < rows->seg_off[r]) return fail(RCP_EINVAL, "seg_off not monotone at row %d", r);
    if (reads->n < 0 || reads->n >= (int64_t(1) << 31))
        return fail(RCP_EUNSUPPORTED, "read count %lld outside [0, 2^31)", (long long)reads->n);
    auto sh = std::make_unique<rcp_shards>();
    sh->devices.assign(device_ids, device_ids + n_devices);
    // ---- the row table, copied in (chromosome, start) order: the blocks are contiguous in that
    // order, so a block's regions are neighbours on the genome and its reads few, whatever order
    // the caller's table is in (an annotation need not be position-sorted)
    const int64_t n_seg = R > 0 ? rows->seg_off[R] : 0;
    sh->n_rows = R;
    std::vector<int32_t> ord((size_t)R);
    for (int32_t r = 0; r < R; ++r) ord[r] = r;
    if (n_devices > 1) {  // (one device: one block, the caller's order)
        // key: the row's first segment's chromosome (an absent one -- NA, outside the readset's
        // codes -- last) and its segments' lowest start
        std::vector<std::pair<int64_t, int64_t>> key((size_t)R);
        for (int32_t r = 0; r < R; ++r) {
            int64_t c = INT64_MAX, lo = INT64_MAX;
            if (rows->seg_off[r + 1] > rows->seg_off[r]) {
                const int32_t c0 = rows->seg_chrom[rows->seg_off[r]];
                c = (c0 >= 0 && c0 < reads->n_chrom) ? c0 : INT64_MAX;
                for (int64_t j = rows->seg_off[r]; j < rows->seg_off[r + 1]; ++j) lo = std::min<int64_t>(lo, rows->seg_start[j]);
            }
            key[r] = {c, lo};
        }
        std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return key[a] < key[b]; });
    }
    bool identity = true;
    for (int32_t r = 0; r < R && identity; ++r) identity = ord[r] == r;
    if (!identity) sh->order = ord;
    sh->seg_off.assign(1, 0);
    sh->chrom.reserve(n_seg);
    for (int32_t i = 0; i < R; ++i) {
        const int32_t r = ord[i];
        const int64_t a = rows->seg_off[r], z = rows->seg_off[r + 1];
        sh->chrom.insert(sh->chrom.end(), rows->seg_chrom + a, rows->seg_chrom + z);
        sh->start.insert(sh->start.end(), rows->seg_start + a, rows->seg_start + z);
        sh->end.insert(sh->end.end(), rows->seg_end + a, rows->seg_end + z);
        sh->strand.insert(sh->strand.end(), rows->seg_strand + a, rows->seg_strand + z);
        if (rows->seg_group) sh->group.insert(sh->group.end(), rows->seg_group + a, rows->seg_group + z);
        sh->seg_off.push_back(sh->seg_off.back() + (z - a));
    }
    if (rows->seg_group) sh->has_group = true;
    if (rows->group_is_list) {
        std::memcpy(sh->is_list, rows->group_is_list, 4);
        sh->has_list = true;
    }
    sh->ignore_strand = rows->ignore_strand ? 1 : 0;
    const bool merged = sh->ignore_strand != 0;
    const int layout = merged ? kLayMerged : kLayStranded;  // the one the row table searches
    const int N = n_devices;
    sh->rs.assign(N, nullptr);
    if (N == 1) {
        // one device: its readset is the whole sample's
        rcp_reads_desc d = *reads;
        d.device = device_ids[0];
        const int rc = readset_build(&d, nullptr, layout, &sh->rs[0]);
        if (rc) return rc;
        sh->split = {0, R};
        *out = sh.release();
        return RCP_OK;
    }
    // ---- A: slices of the reads, one per GPU (device-resident input: one slice, on its device)
    const int K = reads->on_device ? 1 : N;
    std::vector<int32_t> slice_dev(K);
    for (int i = 0; i < K; ++i) slice_dev[i] = reads->on_device ? reads->device : device_ids[i];
    std::vector<rcp_readset*> slice(K, nullptr);
    struct SliceGuard {
        std::vector<rcp_readset*>& v;
        ~SliceGuard() {
            for (rcp_readset*& r : v) {
                rcp_readset_destroy(r);
                r = nullptr;
            }
        }
    } slice_guard{slice};
    const int64_t n = reads->n;
    int rc = run_per_device(K, [&](int i) {
        const int64_t a = n * i / K, b = n * (i + 1) / K;
        ReadSlice sl;
        slice_reads(reads, a, b, &sl);
        sl.d.device = slice_dev[i];
        return readset_build(&sl.d, nullptr, layout | kLayIndexOnly, &slice[i]);
    });
    if (rc) return rc;
    // ---- B: candidate reads of every (range, stream) in every slice
    const rcp_rows_desc all = sh->rows();
    std::vector<std::vector<uint2>> bounds(K);
    rc = run_per_device(K, [&](int i) { return seg_bounds(slice[i], &all, &bounds[i]); });
    if (rc) return rc;
    // row weights: candidates over all slices (the reads the row's pileup streams) + length / 8
    // (its output) + a constant; contiguous blocks in the caller's row order
    std::vector<double> cum((size_t)R + 1, 0.0);
    for (int32_t r = 0; r < R; ++r) {
        double w = 16.0;
        for (int64_t j = sh->seg_off[r]; j < sh->seg_off[r + 1]; ++j) {
            for (int i = 0; i < K; ++i)
                for (int k = 0; k < 3; ++k) w += (double)(bounds[i][3 * j + k].y - bounds[i][3 * j + k].x);
            w += std::max<double>(0.0, (double)sh->end[j] - sh->start[j] + 1) / 8.0;
        }
        cum[r + 1] = cum[r] + w;
    }
    sh->split = balanced_split(cum, N);
    // per (slice i, block b): the candidate ranges of the block's rows in slice i's layout, merged
    // where they overlap or touch inside one stream (a read goes to a block once)
    std::vector<std::vector<std::vector<Range>>> ranges(K, std::vector<std::vector<Range>>(N));
    std::vector<std::vector<int64_t>> cnt(K, std::vector<int64_t>(N, 0));
    rc = run_per_device(K, [&](int i) {
        const ReadLayout& L = merged ? slice[i]->merged : slice[i]->stranded;
        for (int b = 0; b < N; ++b) {
            std::vector<Range> v;
            for (int64_t j = sh->seg_off[sh->split[b]]; j < sh->seg_off[sh->split[b + 1]]; ++j)
                for (int k = 0; k < 3; ++k) {
                    const uint2 x = bounds[i][3 * j + k];
                    if (x.y > x.x) v.push_back(Range{(int32_t)((int64_t)sh->chrom[j] * 3 + k), x.x, x.y});
                }
            auto less = [](const Range& p, const Range& q) { return p.lo < q.lo || (p.lo == q.lo && p.hi < q.hi); };
            if (!std::is_sorted(v.begin(), v.end(), less)) std::sort(v.begin(), v.end(), less);
            std::vector<Range>& m = ranges[i][b];
            for (const Range& x : v) {
                // (ranges of different streams never overlap: streams are disjoint index ranges)
                if (!m.empty() && m.back().sid == x.sid && x.lo <= m.back().hi) m.back().hi = std::max(m.back().hi, x.hi);
                else m.push_back(x);
            }
            int64_t c = 0;
            for (const Range& x : m) {
                if ((int64_t)x.hi > L.h_stream_off[x.sid + 1] || (int64_t)x.lo < L.h_stream_off[x.sid])
                    return fail(RCP_EINVAL, "internal: candidate range outside its stream");
                c += x.hi - x.lo;
            }
            cnt[i][b] = c;
        }
        return (int)RCP_OK;
    });
    if (rc) return rc;
    // ---- C: every block's reads, gathered on the slices' GPUs and copied into the block's GPU
    std::vector<int64_t> n_blk(N, 0);
    for (int b = 0; b < N; ++b)
        for (int i = 0; i < K; ++i) n_blk[b] += cnt[i][b];
    for (int b = 0; b < N; ++b)
        if (n_blk[b] >= (int64_t(1) << 31)) return fail(RCP_EUNSUPPORTED, "block %d holds %lld reads", b, (long long)n_blk[b]);
    std::vector<DevBuf> rcv(N);  // per block: chrom, start, end (int32 each), strand (int8)
    rc = run_per_device(N, [&](int b) {
        DeviceGuard g(device_ids[b]);
        HIP_TRY(g.err);
        const size_t m = (size_t)std::max<int64_t>(n_blk[b], 1);
        HIP_TRY(rcv[b].alloc(13 * m));
        // ignore.strand = TRUE never reads the strand: every read '*'
        if (merged) {
            HIP_TRY(hipMemsetAsync(rcv[b].as<char>() + 12 * m, RCP_STRAND_ANY, m, nullptr));
            HIP_TRY(hipStreamSynchronize(nullptr));  // (the gathers run on non-blocking streams)
        }
        return (int)RCP_OK;
    });
    if (rc) return rc;
    std::vector<int32_t> all_devs(device_ids, device_ids + N);
    for (int32_t d : slice_dev) all_devs.push_back(d);
    enable_peers(all_devs);
    rc = run_per_device(K, [&](int i) {
        DeviceGuard g(slice_dev[i]);
        HIP_TRY(g.err);
        const ReadLayout& L = merged ? slice[i]->merged : slice[i]->stranded;
        // the range table of all blocks, end to end: out_off (int64, n + 1) | lo (uint32) | sid (int32)
        std::vector<int64_t> off(1, 0);
        std::vector<uint32_t> lo;
        std::vector<int32_t> sid;
        std::vector<int64_t> blk0(N + 1, 0);
        for (int b = 0; b < N; ++b) {
            for (const Range& x : ranges[i][b]) {
                off.push_back(off.back() + (x.hi - x.lo));
                lo.push_back(x.lo);
                sid.push_back(x.sid);
            }
            blk0[b + 1] = off.back();
        }
        const int64_t nr = (int64_t)lo.size(), tot = off.back();
        if (tot == 0) return (int)RCP_OK;
        hipStream_t s = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        std::unique_ptr<std::remove_pointer<hipStream_t>::type, hipError_t (*)(hipStream_t)> sguard(s, hipStreamDestroy);
        DevBuf tab, snd;
        HIP_TRY(tab.alloc(8 * (size_t)(nr + 1) + 8 * (size_t)nr));
        int64_t* d_off = tab.as<int64_t>();
        uint32_t* d_lo = reinterpret_cast<uint32_t*>(d_off + nr + 1);
        int32_t* d_sid = reinterpret_cast<int32_t*>(d_lo + nr);
        HIP_TRY(hipMemcpyAsync(d_off, off.data(), 8 * (size_t)(nr + 1), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_lo, lo.data(), 4 * (size_t)nr, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_sid, sid.data(), 4 * (size_t)nr, hipMemcpyHostToDevice, s));
        const size_t t = (size_t)tot;
        HIP_TRY(snd.alloc(13 * t));
        int32_t* sc = snd.as<int32_t>();
        int8_t* sst = reinterpret_cast<int8_t*>(sc + 3 * t);
        HIP_TRY(rcp_launch_gather(tot, nr, d_off, d_lo, d_sid, L.se.as<int2>(), sc, sc + t, sc + 2 * t,
                                  merged ? nullptr : sst, s));
        // block b's part of this slice -> its GPU, after the slices before this one
        for (int b = 0; b < N; ++b) {
            const int64_t c = blk0[b + 1] - blk0[b];
            if (c == 0) continue;
            int64_t at = 0;
            for (int i2 = 0; i2 < i; ++i2) at += cnt[i2][b];
            const size_t m = (size_t)std::max<int64_t>(n_blk[b], 1);
            int32_t* rc32 = rcv[b].as<int32_t>();
            int8_t* rst = reinterpret_cast<int8_t*>(rc32 + 3 * m);
            const int dd = device_ids[b], sd = slice_dev[i];
            for (int q = 0; q < 3; ++q)
                HIP_TRY(hipMemcpyPeerAsync(rc32 + q * m + at, dd, sc + q * t + blk0[b], sd, 4 * (size_t)c, s));
            if (!merged) HIP_TRY(hipMemcpyPeerAsync(rst + at, dd, sst + blk0[b], sd, (size_t)c, s));
        }
        HIP_TRY(hipStreamSynchronize(s));
        return (int)RCP_OK;
    });
    if (rc) return rc;
    for (rcp_readset*& r : slice) {  // the slices' memory is free before the blocks build
        rcp_readset_destroy(r);
        r = nullptr;
    }
    // ---- D: each block's readset from the reads it received (already strand-filtered)
    rc = run_per_device(N, [&](int b) {
        const size_t m = (size_t)std::max<int64_t>(n_blk[b], 1);
        int32_t* rc32 = rcv[b].as<int32_t>();
        rcp_reads_desc d{};
        d.n = n_blk[b];
        d.chrom = rc32;
        d.start = rc32 + m;
        d.end = rc32 + 2 * m;
        d.strand = reinterpret_cast<const int8_t*>(rc32 + 3 * m);
        d.n_chrom = reads->n_chrom;
        d.seqlen = reads->seqlen;
        d.device = device_ids[b];
        d.on_device = 1;
        d.strand_filter = -1;
        const int e = readset_build(&d, nullptr, layout, &sh->rs[b]);
        DeviceGuard g(device_ids[b]);
        rcv[b].reset();
        return e;
    });
    if (rc) return rc;
    *out = sh.release();
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_shards_info(const rcp_shards* sh, int32_t* n_rows, int32_t* n_devices, int32_t* row_split,
                               int64_t* n_reads) {
    RCP_TRY
    if (!sh) return fail(RCP_EINVAL, "NULL shards");
    const int N = (int)sh->devices.size();
    if (n_rows) *n_rows = sh->n_rows;
    if (n_devices) *n_devices = N;
    if (row_split) std::copy(sh->split.begin(), sh->split.end(), row_split);
    if (n_reads)
        for (int b = 0; b < N; ++b) n_reads[b] = sh->rs[b] ? sh->rs[b]->n : 0;
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_shards_rows(const rcp_shards* sh, int32_t* order) {
    RCP_TRY
    if (!sh || !order) return fail(RCP_EINVAL, "NULL argument");
    for (int32_t i = 0; i < sh->n_rows; ++i) order[i] = sh->order.empty() ? i : sh->order[i];
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_shards_profile(rcp_shards* sh, const rcp_bins_desc* bins, double* out, uint8_t* row_valid) {
    RCP_TRY
    if (!sh || !bins) return fail(RCP_EINVAL, "NULL argument");
    const int N = (int)sh->devices.size();
    std::vector<int64_t> n_cols(N, -1);
    const int rc = run_per_device(N, [&](int b) {
        const rcp_rows_desc sub = sh->block(b);
        if (sub.n_rows == 0) return (int)RCP_OK;
        return profile_block(sh->rs[b], &sub, bins, out, sh->n_rows, sh->split[b], row_valid, &n_cols[b], nullptr,
                             sh->order.empty() ? nullptr : sh->order.data() + sh->split[b]);
    });
    if (rc) return rc;
    int64_t nc = -1;
    for (int b = 0; b < N; ++b) {
        if (n_cols[b] < 0) continue;
        if (nc >= 0 && n_cols[b] != nc) return fail(RCP_EINVAL, "row blocks disagree on the column count");
        nc = n_cols[b];
    }
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_shards_coverage(rcp_shards* sh, rcp_cov** out) {
    RCP_TRY
    if (!sh || !out) return fail(RCP_EINVAL, "NULL argument");
    *out = nullptr;
    const int N = (int)sh->devices.size();
    auto res = std::make_unique<rcp_cov>();
    res->n_rows = sh->n_rows;
    res->device = sh->devices[0];
    res->split = sh->split;
    res->order = sh->order;
    std::vector<rcp_cov*> parts(N, nullptr);
    const int rc = run_per_device(N, [&](int b) {
        const rcp_rows_desc sub = sh->block(b);
        return rcp_coverage_rle(sh->rs[b], &sub, &parts[b]);
    });
    for (int b = 0; b < N; ++b) {
        res->parts.emplace_back(parts[b]);
        if (parts[b]) res->n_runs += parts[b]->n_runs;
    }
    if (rc) {
        rcp_cov_free(res.release());
        return rc;
    }
    *out = res.release();
    return RCP_OK;
    RCP_CATCH
}

extern "C" int rcp_shards_destroy(rcp_shards* sh) {
    RCP_TRY
    delete sh;
    return RCP_OK;
    RCP_CATCH
}
