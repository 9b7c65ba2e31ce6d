/*
 * rcp_oracle.c -- CPU ORACLE (test infrastructure only; see rcp_oracle.h header).
 *
 * Restates, per region and in the reference's own dataflow order:
 *   coverageFromRanges  R/coverage.R:176-226
 *   binCoverageMatrix   R/profile.R:153-212  / baseCoverageMatrix R/profile.R:100-151
 *   splitVector         R/util.R:15-85
 * and the upstream primitives those call:
 *   R RNG: set.seed -> Mersenne-Twister (R src/main/RNG.c), sample.int without
 *          replacement (src/main/random.c do_sample), R_unif_index (rejection /
 *          rounding sample.kind);
 *   stats::spline(method = "fmm") (src/library/stats/src/splines.c) + seq.int;
 *   base::mean (long-double two-pass), median.default.
 * Overlaps use a per-chromosome start-sorted copy + max-width window (not the
 * product's prefix-max-end index), so the two implementations are independent.
 */
#include "rcp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* R RNG: Mersenne-Twister exactly as R seeds and tempers it                  */
/* ------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397
typedef struct {
    uint32_t dummy[MT_N + 1]; /* dummy[0] = mti, mt = dummy + 1 (RNG.c) */
} rng_state;

static __thread rng_state g_rng;

static void rng_set_seed(rng_state* s, uint32_t seed) {
    /* RNG_Init: initial scrambling, then fill i_seed[0..624] with the LCG */
    for (int j = 0; j < 50; j++) seed = (69069u * seed + 1u);
    for (int j = 0; j < MT_N + 1; j++) {
        seed = (69069u * seed + 1u);
        s->dummy[j] = seed;
    }
    /* FixupSeeds(MERSENNE_TWISTER, initial = 1): dummy[0] = mti = N */
    s->dummy[0] = MT_N;
}

static double mt_genrand(rng_state* s) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t* mt = s->dummy + 1;
    uint32_t mti = s->dummy[0];
    uint32_t y;
    if (mti >= MT_N) {
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
        mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1];
        mti = 0;
    }
    y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    s->dummy[0] = mti;
    return (double)y * 2.3283064365386963e-10; /* reals: [0,1)-interval */
}

static double unif_rand(rng_state* s) {
    /* fixup(): keep the value in the open interval (0,1) */
    const double i2_32m1 = 2.328306437080797e-10;
    double v = mt_genrand(s);
    if (v <= 0.0) return 0.5 * i2_32m1;
    if (1.0 - v <= 0.0) return 1.0 - 0.5 * i2_32m1;
    return v;
}

static double rbits(rng_state* s, int bits) {
    int64_t v = 0;
    for (int n = 0; n <= bits; n += 16) {
        int v1 = (int)floor(unif_rand(s) * 65536);
        v = 65536 * v + v1;
    }
    const int64_t one64 = 1;
    return (double)(v & ((one64 << bits) - 1));
}

static double unif_index(rng_state* s, double dn, int kind) {
    if (kind == ORC_RNG_ROUNDING) return floor(dn * unif_rand(s));
    if (dn <= 0) return 0.0;
    int bits = (int)ceil(log2(dn));
    double dv;
    do {
        dv = rbits(s, bits);
    } while (dn <= dv);
    return dv;
}

/* sample.int(n, k) without replacement (do_sample), 1-based results. */
static int sample_int(rng_state* s, int n, int k, int kind, int* out, int* work) {
    if (k < 0 || k > n) return -1; /* R: "cannot take a sample larger than the population" */
    for (int i = 0; i < n; i++) work[i] = i;
    int m = n;
    for (int i = 0; i < k; i++) {
        int j = (int)unif_index(s, (double)m, kind);
        out[i] = work[j] + 1;
        work[j] = work[--m];
    }
    return 0;
}

void orc_set_seed(uint32_t seed) { rng_set_seed(&g_rng, seed); }
double orc_unif_rand(void) { return unif_rand(&g_rng); }
int orc_sample(int n, int k, int kind, int* out) {
    int* work = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    int rc = sample_int(&g_rng, n, k, kind, out, work);
    free(work);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* stats::spline, method "fmm" (Forsythe, Malcolm & Moler)                    */
/* ------------------------------------------------------------------------- */
static void fmm_spline(int n, const double* x0, const double* y0, double* b0, double* c0, double* d0) {
    const double* x = x0 - 1;
    const double* y = y0 - 1;
    double *b = b0 - 1, *c = c0 - 1, *d = d0 - 1;
    double t;
    if (n < 2) return;
    if (n < 3) {
        t = (y[2] - y[1]);
        b[1] = t / (x[2] - x[1]);
        b[2] = b[1];
        c[1] = c[2] = d[1] = d[2] = 0.0;
        return;
    }
    const int nm1 = n - 1;
    int i;
    d[1] = x[2] - x[1];
    c[2] = (y[2] - y[1]) / d[1];
    for (i = 2; i < n; i++) {
        d[i] = x[i + 1] - x[i];
        b[i] = 2.0 * (d[i - 1] + d[i]);
        c[i + 1] = (y[i + 1] - y[i]) / d[i];
        c[i] = c[i + 1] - c[i];
    }
    b[1] = -d[1];
    b[n] = -d[nm1];
    c[1] = c[n] = 0.0;
    if (n > 3) {
        c[1] = c[3] / (x[4] - x[2]) - c[2] / (x[3] - x[1]);
        c[n] = c[nm1] / (x[n] - x[n - 2]) - c[n - 2] / (x[nm1] - x[n - 3]);
        c[1] = c[1] * d[1] * d[1] / (x[4] - x[1]);
        c[n] = -c[n] * d[nm1] * d[nm1] / (x[n] - x[n - 3]);
    }
    for (i = 2; i <= n; i++) {
        t = d[i - 1] / b[i - 1];
        b[i] = b[i] - t * d[i - 1];
        c[i] = c[i] - t * c[i - 1];
    }
    c[n] = c[n] / b[n];
    for (i = nm1; i >= 1; i--) c[i] = (c[i] - d[i] * c[i + 1]) / b[i];
    b[n] = (y[n] - y[n - 1]) / d[n - 1] + d[n - 1] * (c[n - 1] + 2.0 * c[n]);
    for (i = 1; i <= nm1; i++) {
        b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i]);
        d[i] = (c[i + 1] - c[i]) / d[i];
        c[i] = 3.0 * c[i];
    }
    c[n] = 3.0 * c[n];
    d[n] = d[nm1];
}

static void spline_eval(int nu, const double* u, double* v, int n, const double* x, const double* y,
                        const double* b, const double* c, const double* d) {
    const int n_1 = n - 1;
    int i = 0;
    for (int l = 0; l < nu; l++) {
        double ul = u[l];
        if (ul < x[i] || (i < n_1 && x[i + 1] < ul)) {
            i = 0;
            int j = n;
            do {
                int k = (i + j) / 2;
                if (ul < x[k]) j = k; else i = k;
            } while (j > i + 1);
        }
        double dx = ul - x[i];
        v[l] = y[i] + dx * (b[i] + dx * (c[i] + dx * d[i]));
    }
}

/* seq.int(from, to, length.out = n) as do_seq computes it. */
static void seq_len_out(double from, double to, int n, double* out) {
    if (n > 0) out[0] = from;
    if (n > 1) out[n - 1] = to;
    if (n > 2) {
        double by = (to - from) / (double)(n - 1);
        for (int i = 1; i < n - 1; i++)
            out[i] = (i < n / 2) ? from + (double)i * by : to - (double)(n - 1 - i) * by;
    }
}

int orc_spline(const double* y, int64_t L, int n, double* out) {
    if (L < 1 || n < 1) return -1;
    double* x = (double*)malloc(sizeof(double) * (size_t)L * 4 + sizeof(double) * (size_t)n);
    double *b = x + L, *c = b + L, *d = c + L, *u = d + L;
    for (int64_t i = 0; i < L; i++) {
        x[i] = (double)(i + 1);
        b[i] = c[i] = d[i] = 0.0;
    }
    fmm_spline((int)L, x, y, b, c, d);
    seq_len_out(1.0, (double)L, n, u);
    spline_eval(n, u, out, (int)L, x, y, b, c, d);
    free(x);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* base::mean / median.default on doubles                                     */
/* ------------------------------------------------------------------------- */
static double r_mean(const double* x, int64_t n) {
    long double s = 0.0L;
    for (int64_t i = 0; i < n; i++) s += x[i];
    s /= n;
    if (isfinite((double)s)) {
        long double t = 0.0L;
        for (int64_t i = 0; i < n; i++) t += (x[i] - s);
        s += t / n;
    }
    return (double)s;
}

static int cmp_double(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static double r_median(const double* x, int64_t n, double* work) {
    for (int64_t i = 0; i < n; i++)
        if (isnan(x[i])) return NAN;
    if (n == 0) return NAN;
    memcpy(work, x, sizeof(double) * (size_t)n);
    qsort(work, (size_t)n, sizeof(double), cmp_double);
    int64_t half = (n + 1) / 2;
    if (n % 2 == 1) return work[half - 1];
    double two[2] = {work[half - 1], work[half]};
    return r_mean(two, 2);
}

/* ------------------------------------------------------------------------- */
/* splitVector (util.R:15-85)                                                 */
/* ------------------------------------------------------------------------- */
static int neighborhood(const double* x, int64_t L, int n, double* y, rng_state* rs, int kind) {
    /* util.R:53-69 (and :21-39 for auto).  Only the index patterns R evaluates
     * without error for L >= 4 are restated; smaller L is reported as an error. */
    if (L < 4 || n < 5) return -2;
    double* pre = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; i++) pre[i] = NAN;
    rng_set_seed(rs, 42);
    pre[0] = x[0];
    pre[1] = x[1];
    pre[n - 2] = x[L - 2];
    pre[n - 1] = x[L - 1];
    int k = (int)(L - 4);
    int pool = n - 4; /* length(3:(n-2)) */
    int* pos = (int*)malloc(sizeof(int) * (size_t)(k > 0 ? k : 1));
    int* work = (int*)malloc(sizeof(int) * (size_t)(pool > 3 ? pool : 3));
    int rc;
    if (pool == 1) {
        /* sample(3, k): a length-one numeric x >= 1 means sample.int(3, k) */
        rc = sample_int(rs, 3, k, kind, pos, work);
    } else {
        rc = sample_int(rs, pool, k, kind, pos, work);
        for (int i = 0; i < k; i++) pos[i] += 2; /* x[idx] with x = 3:(n-2) */
    }
    if (rc != 0) {
        free(pre); free(pos); free(work);
        return -3;
    }
    /* sort(orig.pos) */
    for (int i = 1; i < k; i++) {
        int v = pos[i], j = i - 1;
        while (j >= 0 && pos[j] > v) { pos[j + 1] = pos[j]; j--; }
        pos[j + 1] = v;
    }
    for (int i = 0; i < k; i++) pre[pos[i] - 1] = x[2 + i]; /* y[orig.pos] <- x[3:(L-2)] */
    for (int z = 0; z < n; z++) {
        if (!isnan(pre[z])) {
            y[z] = pre[z];
            continue;
        }
        /* mean(yy[c(z-2,z-1,z+1,z+2)], na.rm = TRUE) over the pre-fill vector */
        double v[4];
        int m = 0;
        int nb[4] = {z - 2, z - 1, z + 1, z + 2};
        for (int q = 0; q < 4; q++)
            if (nb[q] >= 0 && nb[q] < n && !isnan(pre[nb[q]])) v[m++] = pre[nb[q]];
        y[z] = m ? r_mean(v, m) : NAN;
    }
    free(pre); free(pos); free(work);
    return 0;
}

int orc_split_vector(const double* x_in, int64_t L, int n, int interp, int stat, int kind,
                     double* out, int64_t* out_len) {
    rng_state* rs = &g_rng;
    if (n < 1) return -1;
    const double* x = x_in;
    double* tmp = NULL;
    int64_t len = L;
    if (L < n) {
        int mode = interp;
        if (mode == ORC_INTERP_AUTO) mode = ((double)(n - L) / n < 0.2) ? ORC_INTERP_NEIGHBORHOOD : ORC_INTERP_SPLINE;
        if (mode == ORC_INTERP_SPLINE) {
            if (L < 1) return -4;
            tmp = (double*)malloc(sizeof(double) * (size_t)n);
            orc_spline(x_in, L, n, tmp);
            for (int i = 0; i < n; i++)
                if (tmp[i] < 0) tmp[i] = 0; /* x[x<0] <- 0 */
            x = tmp;
            len = n;
        } else if (mode == ORC_INTERP_NEIGHBORHOOD) {
            tmp = (double*)malloc(sizeof(double) * (size_t)n);
            int rc = neighborhood(x_in, L, n, tmp, rs, kind);
            if (rc) {
                free(tmp);
                return rc;
            }
            x = tmp;
            len = n;
        }
        /* ORC_INTERP_LINEAR: the switch arm is spelled "inear" (util.R:49), so
         * "linear" matches nothing and x stays as it is. */
    }
    int64_t bs = len / n;
    int64_t dif = len - bs * n;
    int64_t* size = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    int* add = (int*)malloc(sizeof(int) * (size_t)(dif > 0 ? dif : 1));
    int* work = (int*)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; i++) size[i] = bs;
    rng_set_seed(rs, 42);
    sample_int(rs, n, (int)dif, kind, add, work);
    for (int64_t i = 0; i < dif; i++) size[add[i] - 1] += 1;
    double* w = (double*)malloc(sizeof(double) * (size_t)(bs + 2));
    int64_t pos = 0, k = 0;
    for (int i = 0; i < n; i++) {
        if (size[i] == 0) continue; /* empty factor levels vanish from split() */
        out[k++] = (stat == ORC_STAT_MEDIAN) ? r_median(x + pos, size[i], w) : r_mean(x + pos, size[i]);
        pos += size[i];
    }
    *out_len = k;
    free(size); free(add); free(work); free(w); free(tmp);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* splitBySeqname: per-chromosome start-sorted copies                         */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t n;
    int32_t* start;
    int32_t* end;
    int8_t* strand;
    int32_t maxw;
    int64_t seqlen;
} chrom_reads;

struct orc_index {
    int32_t n_chrom;
    chrom_reads* c;
};

typedef struct {
    int32_t s, e;
    int8_t st;
} rd;

static int cmp_rd(const void* a, const void* b) {
    const rd* x = (const rd*)a;
    const rd* y = (const rd*)b;
    if (x->s != y->s) return (x->s > y->s) - (x->s < y->s);
    return (x->e > y->e) - (x->e < y->e);
}

orc_index* orc_index_build(const orc_reads_in* r, int strand_filter) {
    orc_index* ix = (orc_index*)calloc(1, sizeof(orc_index));
    ix->n_chrom = r->n_chrom;
    ix->c = (chrom_reads*)calloc((size_t)r->n_chrom, sizeof(chrom_reads));
    int64_t* cnt = (int64_t*)calloc((size_t)r->n_chrom, sizeof(int64_t));
    for (int64_t i = 0; i < r->n; i++)
        if (strand_filter < 0 || r->strand[i] == strand_filter) cnt[r->chrom[i]]++;
    rd** buf = (rd**)calloc((size_t)r->n_chrom, sizeof(rd*));
    int64_t* fill = (int64_t*)calloc((size_t)r->n_chrom, sizeof(int64_t));
    for (int c = 0; c < r->n_chrom; c++) buf[c] = (rd*)malloc(sizeof(rd) * (size_t)(cnt[c] ? cnt[c] : 1));
    for (int64_t i = 0; i < r->n; i++) {
        if (!(strand_filter < 0 || r->strand[i] == strand_filter)) continue;
        int c = r->chrom[i];
        rd v = {r->start[i], r->end[i], r->strand[i]};
        buf[c][fill[c]++] = v;
    }
    for (int c = 0; c < r->n_chrom; c++) {
        chrom_reads* cr = &ix->c[c];
        int sorted = 1; /* skip the sort for input already in (start, end) order */
        for (int64_t i = 1; i < cnt[c] && sorted; i++) sorted = cmp_rd(&buf[c][i - 1], &buf[c][i]) <= 0;
        if (!sorted) qsort(buf[c], (size_t)cnt[c], sizeof(rd), cmp_rd);
        cr->n = cnt[c];
        cr->start = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cnt[c] ? cnt[c] : 1));
        cr->end = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cnt[c] ? cnt[c] : 1));
        cr->strand = (int8_t*)malloc((size_t)(cnt[c] ? cnt[c] : 1));
        cr->maxw = 0;
        for (int64_t i = 0; i < cnt[c]; i++) {
            cr->start[i] = buf[c][i].s;
            cr->end[i] = buf[c][i].e;
            cr->strand[i] = buf[c][i].st;
            int32_t w = buf[c][i].e - buf[c][i].s + 1;
            if (w > cr->maxw) cr->maxw = w;
        }
        cr->seqlen = r->seqlen ? r->seqlen[c] : -1;
        free(buf[c]);
    }
    free(buf); free(fill); free(cnt);
    return ix;
}

void orc_index_free(orc_index* ix) {
    if (!ix) return;
    for (int c = 0; c < ix->n_chrom; c++) {
        free(ix->c[c].start); free(ix->c[c].end); free(ix->c[c].strand);
    }
    free(ix->c);
    free(ix);
}

static int64_t lower_bound_i32(const int32_t* a, int64_t n, int64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t m = (lo + hi) / 2;
        if ((int64_t)a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

static int strand_compatible(int8_t q, int8_t s) { return q == 2 || s == 2 || q == s; }

/* i2k length: R's s:e counts |e - s| + 1 elements, index 0 is dropped. */
static int64_t seq_count(int64_t s, int64_t e, int* has_neg) {
    int64_t lo = s < e ? s : e, hi = s < e ? e : s;
    int64_t n = hi - lo + 1;
    if (lo <= 0 && hi >= 0) n -= 1;
    if (lo < 0) *has_neg = 1;
    return n;
}

static int64_t nominal_length(const orc_mask_in* m, int32_t r, int* has_neg) {
    int64_t L = 0;
    for (int64_t j = m->seg_off[r]; j < m->seg_off[r + 1]; j++) L += seq_count(m->seg_start[j], m->seg_end[j], has_neg);
    return L;
}

/* coverageFromRanges for one mask element.  Returns the coverage length, or -1 for
 * the reference's NULL.  out (capacity = nominal length) receives the depth. */
static int64_t coverage_one(const orc_index* ix, const orc_mask_in* m, int32_t r, int ignore_strand,
                            int32_t* out) {
    int64_t j0 = m->seg_off[r], j1 = m->seg_off[r + 1];
    if (j1 <= j0) return -1;
    int32_t chr = m->seg_chrom[j0];
    if (chr < 0 || chr >= ix->n_chrom || ix->c[chr].n == 0) return -1; /* "not found!" */
    const chrom_reads* cr = &ix->c[chr];
    /* findOverlaps(x, reads) -> subjectHits (one entry per (segment, read) pair) */
    int64_t cap = 1024, nh = 0;
    int64_t* hits = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    for (int64_t j = j0; j < j1; j++) {
        int64_t qs = m->seg_start[j], qe = m->seg_end[j];
        if (qe < qs) continue; /* zero-width query: no overlaps (documented) */
        int64_t i = lower_bound_i32(cr->start, cr->n, qs - cr->maxw + 1);
        for (; i < cr->n && cr->start[i] <= qe; i++) {
            if (cr->end[i] < qs) continue;
            if (!ignore_strand && !strand_compatible(m->seg_strand[j], cr->strand[i])) continue;
            if (nh == cap) {
                cap *= 2;
                hits = (int64_t*)realloc(hits, sizeof(int64_t) * (size_t)cap);
            }
            hits[nh++] = i;
        }
    }
    if (nh == 0) {
        free(hits);
        return -1; /* length(y$reads) == 0 -> NULL */
    }
    /* coverage(y$reads)[[cc]]: Rle of length seqlength, or max end of the hits when NA */
    int64_t rle_len = cr->seqlen;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t h = 0; h < nh; h++) {
        if (cr->end[hits[h]] > hi) hi = cr->end[hits[h]];
        if (cr->start[hits[h]] < lo) lo = cr->start[hits[h]];
    }
    if (rle_len < 0) rle_len = hi;
    /* subscript checks: [i2k] errors on mixed signs or an index beyond the Rle */
    int has_neg = 0;
    int64_t plo = INT64_MAX, phi = INT64_MIN;
    for (int64_t j = j0; j < j1; j++) {
        int64_t s = m->seg_start[j], e = m->seg_end[j];
        int64_t a = s < e ? s : e, b = s < e ? e : s;
        if (a < 0) has_neg = 1;
        if (a < plo) plo = a;
        if (b > phi) phi = b;
    }
    if (has_neg || phi > rle_len) {
        free(hits);
        return -1; /* tryCatch(error) -> NULL */
    }
    if (plo < 1) plo = 1;
    /* depth over the span [plo, phi] by a difference array */
    int64_t span = phi - plo + 1;
    int32_t* dep = (int32_t*)calloc((size_t)span + 1, sizeof(int32_t));
    for (int64_t h = 0; h < nh; h++) {
        int64_t a = cr->start[hits[h]], b = cr->end[hits[h]];
        if (b < plo || a > phi) continue;
        if (a < plo) a = plo;
        if (b > phi) b = phi;
        dep[a - plo] += 1;
        dep[b - plo + 1] -= 1;
    }
    for (int64_t p = 1; p < span; p++) dep[p] += dep[p - 1];
    int64_t k = 0;
    for (int64_t j = j0; j < j1; j++) {
        int64_t s = m->seg_start[j], e = m->seg_end[j];
        int64_t step = (e >= s) ? 1 : -1;
        for (int64_t p = s;; p += step) {
            if (p != 0) out[k++] = dep[p - plo];
            if (p == e) break;
        }
    }
    free(dep);
    free(hits);
    if (m->seg_strand[j0] == 1) { /* rev() for '-' */
        for (int64_t a = 0, b = k - 1; a < b; a++, b--) {
            int32_t t = out[a];
            out[a] = out[b];
            out[b] = t;
        }
    }
    return k;
}

/* ------------------------------------------------------------------------- */
/* cmclapply stand-in: a pthread pool over regions                            */
/* ------------------------------------------------------------------------- */
typedef struct {
    void (*fn)(void* ctx, int32_t r);
    void* ctx;
    int32_t n;
    int32_t next;
    pthread_mutex_t mu;
} pool_t;

static void* pool_worker(void* arg) {
    pool_t* p = (pool_t*)arg;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        int32_t r0 = p->next;
        p->next += 16;
        pthread_mutex_unlock(&p->mu);
        if (r0 >= p->n) break;
        int32_t r1 = r0 + 16 < p->n ? r0 + 16 : p->n;
        for (int32_t r = r0; r < r1; r++) p->fn(p->ctx, r);
    }
    return NULL;
}

static void parallel_for(int32_t n, int nthreads, void (*fn)(void*, int32_t), void* ctx) {
    if (nthreads <= 1) {
        for (int32_t r = 0; r < n; r++) fn(ctx, r);
        return;
    }
    pool_t p = {fn, ctx, n, 0, PTHREAD_MUTEX_INITIALIZER};
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, pool_worker, &p);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
}

typedef struct {
    const orc_index* ix;
    const orc_mask_in* m;
    int ignore_strand;
    const int64_t* off;
    int32_t* cov;
    uint8_t* valid;
    int64_t* len;
} cov_ctx;

static void cov_task(void* c_, int32_t r) {
    cov_ctx* c = (cov_ctx*)c_;
    int64_t L = coverage_one(c->ix, c->m, r, c->ignore_strand, c->cov + c->off[r]);
    c->valid[r] = L >= 0;
    c->len[r] = L >= 0 ? L : 0;
}

int orc_coverage(const orc_index* ix, const orc_mask_in* mask, int ignore_strand, int nthreads,
                 const int64_t* out_off, int32_t* out_cov, uint8_t* valid, int64_t* out_len) {
    if (!out_cov) {
        for (int32_t r = 0; r < mask->n; r++) {
            int neg = 0;
            out_len[r] = nominal_length(mask, r, &neg);
        }
        return 0;
    }
    cov_ctx c = {ix, mask, ignore_strand, out_off, out_cov, valid, out_len};
    parallel_for(mask->n, nthreads, cov_task, &c);
    return 0;
}

typedef struct {
    const orc_index* ix;
    const orc_mask_in* m;
    int ignore_strand;
    double scale;
    int where, f1, f2, n, interp, stat, kind;
    double* out;
    int64_t ncol;
    uint8_t* valid;
    int32_t R;
    volatile int err;
} prof_ctx;

static void prof_task(void* c_, int32_t r) {
    prof_ctx* c = (prof_ctx*)c_;
    int neg = 0;
    int64_t cap = nominal_length(c->m, r, &neg);
    int64_t need = cap > c->ncol ? cap : c->ncol;
    if (need < c->n) need = c->n;
    int32_t* cov = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cap > 0 ? cap : 1));
    double* x = (double*)malloc(sizeof(double) * (size_t)(need + 1));
    double* row = (double*)malloc(sizeof(double) * (size_t)(need + 1));
    int64_t L = coverage_one(c->ix, c->m, r, c->ignore_strand, cov);
    c->valid[r] = L >= 0;
    int64_t rl = 0;
    if (L < 0) {
        /* NULL -> rep(0, binSize) (or rep(0, size) per base) */
        int64_t z = c->n > 0 ? c->n : c->ncol;
        for (int64_t i = 0; i < z; i++) x[i] = 0.0;
        if (c->n > 0) {
            if (orc_split_vector(x, z, c->n, c->interp, c->stat, c->kind, row, &rl)) c->err = 1;
        } else {
            memcpy(row, x, sizeof(double) * (size_t)z);
            rl = z;
        }
    } else {
        /* as.numeric(x) (times the linear normalization factor, recoup.R:559-577) */
        int64_t a = 0, b = L; /* slice [a, b) */
        if (c->where == ORC_WHERE_CENTER) { a = c->f1; b = L - c->f2; }
        else if (c->where == ORC_WHERE_UPSTREAM) { a = 0; b = c->f1; }
        else if (c->where == ORC_WHERE_DOWNSTREAM) { a = L - c->f2; b = L; }
        if (a < 0 || b > L || b < a) {
            c->err = 2;
            rl = 0;
        } else {
            for (int64_t i = a; i < b; i++) x[i - a] = (double)cov[i] * c->scale;
            if (c->n > 0) {
                if (orc_split_vector(x, b - a, c->n, c->interp, c->stat, c->kind, row, &rl)) c->err = 1;
            } else {
                memcpy(row, x, sizeof(double) * (size_t)(b - a));
                rl = b - a;
            }
        }
    }
    /* rbind(): a row shorter than ncol is recycled */
    for (int64_t j = 0; j < c->ncol; j++) c->out[(size_t)j * c->R + r] = rl > 0 ? row[j % rl] : 0.0;
    free(cov); free(x); free(row);
}

int orc_profile(const orc_index* ix, const orc_mask_in* mask, int ignore_strand, double scale,
                int where, int f1, int f2, int n, int interp, int stat, int rng_kind,
                int nthreads, double* out, int64_t ncol, uint8_t* valid) {
    prof_ctx c = {ix, mask, ignore_strand, scale, where, f1, f2, n, interp, stat, rng_kind,
                  out, ncol, valid, mask->n, 0};
    parallel_for(mask->n, nthreads, prof_task, &c);
    return c.err ? -c.err : 0;
}

/* ------------------------------------------------------------------------- */
/* Rows of several mask elements (coverageRnaRef) + several column parts      */
/* ------------------------------------------------------------------------- */
/* A row is c(cov(g0), cov(g1), ...) over its groups (R/coverage.R:101-121: left flank,
 * the gene's exon list, right flank), NULL when any group is NULL; the profile row is
 * cbind over the parts (R/profile.R:13-81): each part slices the row (where, flank) and
 * bins it with splitVector (n_bins > 0) or copies it per base (n_bins == 0); a NULL row
 * gives zeros (rep(0, binSize) binned, rep(0, size) per base). */
typedef struct {
    const orc_index* ix;
    const orc_rows_in* rows;
    const orc_parts_in* parts;
    int ignore_strand;
    double* out;
    uint8_t* valid;
    int64_t ncol;
    volatile int err;
} rows_ctx;

static void rows_task(void* c_, int32_t r) {
    rows_ctx* c = (rows_ctx*)c_;
    const orc_rows_in* R = c->rows;
    const orc_parts_in* P = c->parts;
    const int64_t j0 = R->seg_off[r], j1 = R->seg_off[r + 1];
    int64_t cap = 0;
    {
        orc_mask_in all = {1, NULL, R->seg_chrom + j0, R->seg_start + j0, R->seg_end + j0, R->seg_strand + j0};
        int64_t off[2] = {0, j1 - j0};
        int neg = 0;
        all.seg_off = off;
        cap = nominal_length(&all, 0, &neg);
    }
    int32_t* cov = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cap > 0 ? cap : 1));
    int64_t L = 0;
    int ok = j1 > j0;
    for (int64_t g0 = j0; ok && g0 < j1;) {
        const int grp = R->seg_group ? R->seg_group[g0] : 0;
        int64_t g1 = g0;
        while (g1 < j1 && (R->seg_group ? R->seg_group[g1] : 0) == grp) ++g1;
        /* one mask element: a GRangesList element (all its ranges) or one GRanges range each */
        const int multi = R->group_is_list && R->group_is_list[grp];
        for (int64_t a = g0; ok && a < g1; a = multi ? g1 : a + 1) {
            const int64_t b = multi ? g1 : a + 1;
            int64_t off[2] = {0, b - a};
            orc_mask_in m = {1, off, R->seg_chrom + a, R->seg_start + a, R->seg_end + a, R->seg_strand + a};
            const int64_t k = coverage_one(c->ix, &m, 0, c->ignore_strand, cov + L);
            if (k < 0) ok = 0; else L += k;
        }
        g0 = g1;
    }
    c->valid[r] = (uint8_t)ok;
    int64_t col = 0;
    for (int p = 0; p < P->n_parts; ++p) {
        const int n = P->n_bins[p];
        const int64_t ncol_p = n > 0 ? n : P->per_base_width[p];
        int64_t need = ncol_p > L ? ncol_p : L;
        double* x = (double*)malloc(sizeof(double) * (size_t)(need + 1));
        double* row = (double*)malloc(sizeof(double) * (size_t)(need + 1));
        int64_t rl = 0;
        if (!ok) {
            for (int64_t i = 0; i < ncol_p; i++) x[i] = 0.0;
            if (n > 0) {
                if (orc_split_vector(x, n, n, P->interp, P->stat, P->rng_kind, row, &rl)) c->err = 1;
            } else {
                memcpy(row, x, sizeof(double) * (size_t)ncol_p);
                rl = ncol_p;
            }
        } else {
            int64_t a = 0, b = L;
            const int w = P->where[p];
            if (w == ORC_WHERE_CENTER) { a = P->f1; b = L - P->f2; }
            else if (w == ORC_WHERE_UPSTREAM) { a = 0; b = P->f1; }
            else if (w == ORC_WHERE_DOWNSTREAM) { a = L - P->f2; b = L; }
            if (a < 0 || b > L || b < a) {
                c->err = 2;
            } else {
                for (int64_t i = a; i < b; i++) x[i - a] = (double)cov[i] * P->scale;
                if (n > 0) {
                    if (orc_split_vector(x, b - a, n, P->interp, P->stat, P->rng_kind, row, &rl)) c->err = 1;
                } else {
                    memcpy(row, x, sizeof(double) * (size_t)(b - a));
                    rl = b - a;
                }
            }
        }
        for (int64_t j = 0; j < ncol_p; j++) c->out[(size_t)(col + j) * R->n + r] = rl > 0 ? row[j % rl] : 0.0;
        col += ncol_p;
        free(x);
        free(row);
    }
    free(cov);
}

int orc_profile_rows(const orc_index* ix, const orc_rows_in* rows, const orc_parts_in* parts, int ignore_strand,
                     int nthreads, double* out, uint8_t* valid) {
    rows_ctx c = {ix, rows, parts, ignore_strand, out, valid, 0, 0};
    parallel_for(rows->n, nthreads, rows_task, &c);
    return c.err ? -c.err : 0;
}
