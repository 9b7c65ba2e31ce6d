// rcp_bam.cpp -- BAM ingest for the read sets (readBam, R/ranges.R:111-146).
//
// readGAlignments(file) -> as(., "GRanges") / grglist(.) -> trim(): each mapped alignment
// becomes its reference span [pos + 1, pos + width] (keep), or one range per block between
// N-skips (split), on its reference sequence and strand (flag 0x10), clipped to the
// sequence length.  "remove" drops alignments wider than quantile(width, q) (R type 7).
// BGZF blocks are inflated in parallel (zlib raw deflate), records are decoded on the host
// and handed to rcp_readset_create, which sorts them on the GPU.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/recoup_amd.h"

int rcp_internal_fail(int code, const char* msg);  // rcp_host.cpp: the rcp_last_error() channel

namespace {

int bam_fail(int code, const char* msg) { return rcp_internal_fail(code, msg); }

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
int32_t rd32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24)); }

struct Block {
    size_t off;    // compressed data (deflate stream) offset in the file
    size_t clen;   // deflate bytes
    size_t ulen;   // ISIZE
    size_t uoff;   // offset in the decompressed stream
};

}  // namespace

struct rcp_bam {
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_len;
    std::vector<int32_t> chrom, start, end;
    std::vector<int8_t> strand;
    int64_t n_alignments = 0;  // mapped alignments read
};

namespace {
int bam_read(const char* path, int splice_action, double remove_q, int n_threads, rcp_bam** out);
}

extern "C" int rcp_bam_read(const char* path, int splice_action, double remove_q, int n_threads, rcp_bam** out) {
    // nothing may escape into the caller's process (an R session): every C++ exception
    // becomes an RCP_E* code
    try {
        return bam_read(path, splice_action, remove_q, n_threads, out);
    } catch (const std::bad_alloc&) {
        return bam_fail(RCP_ENOMEM, "host memory exhausted while reading the BAM file");
    } catch (const std::exception& e) {
        return bam_fail(RCP_ESEMANTIC, e.what());
    } catch (...) {
        return bam_fail(RCP_ESEMANTIC, "unexpected error while reading the BAM file");
    }
}

namespace {
int bam_read(const char* path, int splice_action, double remove_q, int n_threads, rcp_bam** out) {
    if (!path || !out) return bam_fail(RCP_EINVAL, "NULL argument");
    *out = nullptr;
    if (splice_action < RCP_SPLICE_KEEP || splice_action > RCP_SPLICE_SPLIT)
        return bam_fail(RCP_EINVAL, "splice_action must be keep, remove or split");
    if (!(remove_q >= 0.0 && remove_q <= 1.0)) return bam_fail(RCP_EINVAL, "spliceRemoveQ outside [0, 1]");
    FILE* f = std::fopen(path, "rb");
    if (!f) return bam_fail(RCP_EINVAL, "cannot open the BAM file");
    std::vector<uint8_t> file;
    {
        std::fseek(f, 0, SEEK_END);
        const long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        if (sz < 0) {
            std::fclose(f);
            return bam_fail(RCP_EINVAL, "cannot size the BAM file");
        }
        file.resize((size_t)sz);
        const size_t got = sz ? std::fread(file.data(), 1, (size_t)sz, f) : 0;
        std::fclose(f);
        if (got != (size_t)sz) return bam_fail(RCP_EINVAL, "short read of the BAM file");
    }
    // ---- BGZF block table (gzip members with the BC extra subfield)
    std::vector<Block> blocks;
    size_t p = 0, total = 0;
    while (p < file.size()) {
        if (file.size() - p < 18) return bam_fail(RCP_ESEMANTIC, "truncated BGZF block header");
        const uint8_t* h = file.data() + p;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return bam_fail(RCP_ESEMANTIC, "not a BGZF file");
        const uint16_t xlen = rd16(h + 10);
        // the extra field must lie inside the file before any subfield is read
        if ((size_t)xlen + 12 > file.size() - p) return bam_fail(RCP_ESEMANTIC, "truncated BGZF extra field");
        int64_t bsize = -1;
        for (size_t x = 12; x + 4 <= 12 + (size_t)xlen;) {
            const uint16_t slen = rd16(h + x + 2);
            if (x + 4 + (size_t)slen > 12 + (size_t)xlen) return bam_fail(RCP_ESEMANTIC, "BGZF subfield beyond XLEN");
            if (h[x] == 66 && h[x + 1] == 67 && slen == 2) bsize = rd16(h + x + 4);
            x += 4 + slen;
        }
        if (bsize < 0) return bam_fail(RCP_ESEMANTIC, "BGZF block without BSIZE");
        const size_t blen = (size_t)bsize + 1;
        if (blen > file.size() - p || blen < (size_t)xlen + 20) return bam_fail(RCP_ESEMANTIC, "truncated BGZF block");
        Block b;
        b.off = p + 12 + xlen;
        b.clen = blen - xlen - 20;
        b.ulen = (size_t)(uint32_t)rd32(file.data() + p + blen - 4);
        // ISIZE of a BGZF block is at most 64 KiB (SAM spec 4.1); larger values are corrupt
        if (b.ulen > 65536) return bam_fail(RCP_ESEMANTIC, "BGZF block ISIZE above 65536");
        b.uoff = total;
        total += b.ulen;
        blocks.push_back(b);
        p += blen;
    }
    // ---- inflate in parallel
    std::vector<uint8_t> data(total);
    std::atomic<size_t> next{0};
    std::atomic<int> bad{0};
    const int nt = std::max(1, std::min(n_threads > 0 ? n_threads : 1, 64));
    auto work = [&]() {
        z_stream z;
        std::memset(&z, 0, sizeof z);
        if (inflateInit2(&z, -15) != Z_OK) {
            bad = 1;
            return;
        }
        for (size_t i; (i = next.fetch_add(1)) < blocks.size();) {
            const Block& b = blocks[i];
            inflateReset(&z);
            z.next_in = file.data() + b.off;
            z.avail_in = (uInt)b.clen;
            z.next_out = data.data() + b.uoff;
            z.avail_out = (uInt)b.ulen;
            const int rc = inflate(&z, Z_FINISH);
            if (rc != Z_STREAM_END || z.avail_out != 0) bad = 1;
        }
        inflateEnd(&z);
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) {
            try {
                th.emplace_back(work);
            } catch (const std::exception&) {
                break;  // fewer threads (the calling one always works)
            }
        }
        work();
        for (auto& t : th) t.join();
    }
    if (bad) return bam_fail(RCP_ESEMANTIC, "corrupt BGZF block");
    file.clear();
    file.shrink_to_fit();
    // ---- header
    const uint8_t* d = data.data();
    const size_t n = data.size();
    if (n < 12 || std::memcmp(d, "BAM\1", 4) != 0) return bam_fail(RCP_ESEMANTIC, "missing BAM magic");
    auto res = new rcp_bam();
    std::unique_ptr<rcp_bam> guard(res);
    size_t o = 4;
    const int32_t l_text = rd32(d + o);
    o += 4 + (size_t)std::max(l_text, 0);
    if (o + 4 > n) return bam_fail(RCP_ESEMANTIC, "truncated BAM header");
    const int32_t n_ref = rd32(d + o);
    o += 4;
    for (int32_t i = 0; i < n_ref; ++i) {
        if (o + 4 > n) return bam_fail(RCP_ESEMANTIC, "truncated reference list");
        const int32_t l_name = rd32(d + o);
        o += 4;
        if (l_name < 1 || o + (size_t)l_name + 4 > n) return bam_fail(RCP_ESEMANTIC, "bad reference name");
        res->ref_names.emplace_back(reinterpret_cast<const char*>(d + o), (size_t)l_name - 1);
        o += (size_t)l_name;
        res->ref_len.push_back(rd32(d + o));
        o += 4;
    }
    // ---- alignments
    std::vector<int32_t> widths;  // trimmed alignment spans (remove)
    while (o + 4 <= n) {
        const int32_t bs = rd32(d + o);
        if (bs < 32 || o + 4 + (size_t)bs > n) return bam_fail(RCP_ESEMANTIC, "truncated alignment record");
        const uint8_t* r = d + o + 4;
        o += 4 + (size_t)bs;
        const int32_t ref = rd32(r);
        const int32_t pos = rd32(r + 4);
        const uint8_t l_read_name = r[8];
        const uint16_t n_cigar = rd16(r + 12);
        const uint16_t flag = rd16(r + 14);
        if ((flag & 0x4) || ref < 0 || ref >= n_ref || pos < 0) continue;  // readGAlignments: mapped only
        if (32 + (size_t)l_read_name + 4 * (size_t)n_cigar > (size_t)bs)
            return bam_fail(RCP_ESEMANTIC, "alignment CIGAR beyond its record");
        const uint8_t* cig = r + 32 + l_read_name;
        const int8_t st = (flag & 0x10) ? 1 : 0;
        const int64_t seqlen = res->ref_len[ref];
        ++res->n_alignments;
        // reference-consuming runs: M D N = X; blocks end at N (grglist, drop.D.ranges = FALSE)
        int64_t x = (int64_t)pos + 1, bstart = x, width = 0;
        auto emit = [&](int64_t a, int64_t b) {  // trim() to [1, seqlength]
            a = std::max<int64_t>(a, 1);
            if (seqlen > 0) b = std::min<int64_t>(b, seqlen);
            res->chrom.push_back(ref);
            res->start.push_back((int32_t)a);
            res->end.push_back((int32_t)std::max<int64_t>(b, a - 1));
            res->strand.push_back(st);
        };
        const size_t before = res->start.size();
        for (uint16_t c = 0; c < n_cigar; ++c) {
            const uint32_t v = (uint32_t)rd32(cig + 4 * c);
            const uint32_t op = v & 15, len = v >> 4;
            const bool ref_op = op == 0 || op == 2 || op == 3 || op == 7 || op == 8;
            if (!ref_op) continue;
            if (op == 3 && splice_action == RCP_SPLICE_SPLIT) {
                if (x > bstart) emit(bstart, x - 1);
                x += len;
                bstart = x;
            } else {
                x += len;
            }
            width += len;
        }
        if (splice_action == RCP_SPLICE_SPLIT) {
            if (x > bstart || res->start.size() == before) emit(bstart, x - 1);
        } else {
            emit((int64_t)pos + 1, (int64_t)pos + std::max<int64_t>(width, 0));
            widths.push_back(res->end.back() - res->start.back() + 1);  // width after trim()
        }
    }
    if (splice_action == RCP_SPLICE_REMOVE && !widths.empty()) {
        // quantile(width(reads), q), type 7: h = (n - 1) q, x[floor h] + (h - floor h)(x[floor h + 1] - x[floor h])
        std::vector<int32_t> sorted(widths);
        std::sort(sorted.begin(), sorted.end());
        const double h = (double)(sorted.size() - 1) * remove_q;
        const size_t lo = (size_t)std::floor(h);
        const size_t hi = std::min(lo + 1, sorted.size() - 1);
        const double qu = sorted[lo] + (h - (double)lo) * (double)(sorted[hi] - sorted[lo]);
        size_t w = 0;
        for (size_t i = 0; i < widths.size(); ++i) {
            if ((double)widths[i] > qu) continue;
            res->chrom[w] = res->chrom[i];
            res->start[w] = res->start[i];
            res->end[w] = res->end[i];
            res->strand[w] = res->strand[i];
            ++w;
        }
        res->chrom.resize(w);
        res->start.resize(w);
        res->end.resize(w);
        res->strand.resize(w);
    }
    *out = guard.release();
    return RCP_OK;
}
}  // namespace

extern "C" int rcp_bam_info(const rcp_bam* b, int64_t* n_reads, int32_t* n_ref, int64_t* n_alignments) {
    if (!b) return bam_fail(RCP_EINVAL, "NULL handle");
    if (n_reads) *n_reads = (int64_t)b->start.size();
    if (n_ref) *n_ref = (int32_t)b->ref_names.size();
    if (n_alignments) *n_alignments = b->n_alignments;
    return RCP_OK;
}

extern "C" const char* rcp_bam_ref_name(const rcp_bam* b, int32_t i) {
    if (!b || i < 0 || i >= (int32_t)b->ref_names.size()) return nullptr;
    return b->ref_names[i].c_str();
}

extern "C" int rcp_bam_copy(const rcp_bam* b, int64_t* ref_len, int32_t* chrom, int32_t* start, int32_t* end,
                            int8_t* strand) {
    if (!b) return bam_fail(RCP_EINVAL, "NULL handle");
    const size_t n = b->start.size();
    if (ref_len) std::copy(b->ref_len.begin(), b->ref_len.end(), ref_len);
    if (n && chrom) std::memcpy(chrom, b->chrom.data(), 4 * n);
    if (n && start) std::memcpy(start, b->start.data(), 4 * n);
    if (n && end) std::memcpy(end, b->end.data(), 4 * n);
    if (n && strand) std::memcpy(strand, b->strand.data(), n);
    return RCP_OK;
}

extern "C" int rcp_bam_free(rcp_bam* b) {
    delete b;
    return RCP_OK;
}
