// abi_driver.cpp -- host-only driver of librecoup_amd's C ABI for the sanitizer build
// (tests/sanitize/Makefile: rcp_host.cpp + rcp_bam.cpp under ASan + UBSan).
//
//   abi_driver bam FILE...   rcp_bam_read every file (all splice actions); print one rc per
//                            file and action; the corpus is truncated / corrupted BAMs
//   abi_driver abi           argument validation of every entry point (NULL handles and
//                            arrays, bad enums) and the R RNG, with no GPU needed
// Any memory error aborts with the sanitizer's report (non-zero exit).
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/recoup_amd.h"

static int bam(int argc, char** argv) {
    for (int i = 2; i < argc; ++i) {
        for (int action = RCP_SPLICE_KEEP; action <= RCP_SPLICE_SPLIT; ++action) {
            rcp_bam* b = nullptr;
            const int rc = rcp_bam_read(argv[i], action, 0.75, 4, &b);
            int64_t n = -1, nal = -1;
            int32_t nref = -1;
            if (rc == RCP_OK) {
                rcp_bam_info(b, &n, &nref, &nal);
                std::vector<int64_t> rl(nref > 0 ? nref : 1);
                std::vector<int32_t> c(n > 0 ? n : 1), s(n > 0 ? n : 1), e(n > 0 ? n : 1);
                std::vector<int8_t> st(n > 0 ? n : 1);
                rcp_bam_copy(b, rl.data(), c.data(), s.data(), e.data(), st.data());
                for (int32_t k = 0; k < nref; ++k) (void)rcp_bam_ref_name(b, k);
                (void)rcp_bam_ref_name(b, -1);
                (void)rcp_bam_ref_name(b, nref);
                rcp_bam_free(b);
            } else if (b != nullptr) {
                std::printf("handle leaked on error\n");
                return 3;
            }
            std::printf("%s %d %d %lld\n", argv[i], action, rc, (long long)n);
        }
    }
    return 0;
}

#define EXPECT(cond)                                              \
    do {                                                          \
        if (!(cond)) {                                            \
            std::printf("FAILED: %s (line %d)\n", #cond, __LINE__); \
            return 1;                                             \
        }                                                         \
    } while (0)

static int abi() {
    EXPECT(std::strlen(rcp_version()) > 0);
    int nd = -1;
    EXPECT(rcp_device_count(&nd) == RCP_OK);
    EXPECT(rcp_device_count(nullptr) == RCP_EINVAL);
    rcp_readset* rs = nullptr;
    rcp_reads_desc d{};
    d.n_chrom = 1;
    EXPECT(rcp_readset_create(nullptr, nullptr, &rs) == RCP_EINVAL);
    EXPECT(rcp_readset_create(&d, nullptr, nullptr) == RCP_EINVAL);
    const int rc = rcp_readset_create(&d, nullptr, &rs);
    EXPECT(nd > 0 ? rc == RCP_OK : rc == RCP_ENODEVICE);
    if (rs) rcp_readset_destroy(rs);
    EXPECT(rcp_readset_info(nullptr, nullptr, nullptr) == RCP_EINVAL);
    rcp_plan* plan = nullptr;
    EXPECT(rcp_plan_create(nullptr, nullptr, nullptr, &plan) == RCP_EINVAL);
    EXPECT(rcp_plan_create_ex(nullptr, nullptr, nullptr, nullptr, &plan) == RCP_EINVAL);
    EXPECT(rcp_plan_destroy(nullptr) == RCP_OK);
    EXPECT(rcp_plan_info_get(nullptr, nullptr) == RCP_EINVAL);
    EXPECT(rcp_plan_execute(nullptr, nullptr, nullptr, nullptr, nullptr) == RCP_EINVAL);
    EXPECT(rcp_plan_status(nullptr, nullptr) == RCP_EINVAL);
    EXPECT(rcp_plan_validity(nullptr, nullptr, nullptr) == RCP_EINVAL);
    EXPECT(rcp_plan_row_lengths(nullptr, nullptr) == RCP_EINVAL);
    EXPECT(rcp_calc_coverage(nullptr, nullptr, nullptr, nullptr, nullptr) == RCP_EINVAL);
    int64_t off[2] = {0, 0}, run_off[2], nruns;
    EXPECT(rcp_rle_encode(-1, off, nullptr, 0, nullptr, nullptr, run_off, &nruns, nullptr) == RCP_EINVAL);
    {  // rcp_profile_rle: host-side validation of the run arrays before any device work
        const int32_t where = RCP_WHERE_WHOLE, nb = 4, w = 0;
        rcp_bins_desc bins{};
        bins.n_parts = 1;
        bins.where = &where;
        bins.n_bins = &nb;
        bins.per_base_width = &w;
        bins.scale = 1.0;
        const int64_t ro[3] = {0, 2, 3};
        const int32_t len_ok[3] = {3, 2, 4}, len_bad[3] = {3, -2, 4}, vals[3] = {1, 0, 5};
        rcp_rle_desc c{2, ro, len_ok, vals, nullptr, nullptr};
        double out[8];
        EXPECT(rcp_profile_rle(nullptr, &bins, 0, out, nullptr) == RCP_EINVAL);
        EXPECT(rcp_profile_rle(&c, nullptr, 0, out, nullptr) == RCP_EINVAL);
        c.lengths = len_bad;
        EXPECT(rcp_profile_rle(&c, &bins, 0, out, nullptr) == RCP_EINVAL);
        const int64_t ro_bad[3] = {0, 3, 2};
        c.lengths = len_ok;
        c.run_off = ro_bad;
        EXPECT(rcp_profile_rle(&c, &bins, 0, out, nullptr) == RCP_EINVAL);
        c.run_off = ro;
        const double dv[3] = {1, 2, 3};
        c.dvalues = dv;  // both value arrays
        EXPECT(rcp_profile_rle(&c, &bins, 0, out, nullptr) == RCP_EINVAL);
        c.dvalues = nullptr;
        const int rc2 = rcp_profile_rle(&c, &bins, 0, out, nullptr);
        EXPECT(nd > 0 ? rc2 == RCP_OK : rc2 == RCP_ENODEVICE);
    }
    EXPECT(rcp_bam_read(nullptr, 0, 0.5, 1, nullptr) == RCP_EINVAL);
    rcp_bam* b = nullptr;
    EXPECT(rcp_bam_read("/nonexistent/x.bam", 0, 0.5, 1, &b) == RCP_EINVAL && b == nullptr);
    EXPECT(rcp_bam_read("/nonexistent/x.bam", 7, 0.5, 1, &b) == RCP_EINVAL);
    EXPECT(rcp_bam_read("/nonexistent/x.bam", 0, 1.5, 1, &b) == RCP_EINVAL);
    EXPECT(rcp_bam_info(nullptr, nullptr, nullptr, nullptr) == RCP_EINVAL);
    // R RNG: set.seed(42); sample(1:10) under both sample.kind values (Appendix B)
    const int64_t rej[10] = {1, 5, 10, 8, 2, 4, 6, 9, 7, 3};
    rcp_rng* g = nullptr;
    EXPECT(rcp_rng_create(42, 5, &g) == RCP_EINVAL);
    EXPECT(rcp_rng_create(42, RCP_RNG_REJECTION, &g) == RCP_OK);
    int64_t s[10];
    EXPECT(rcp_rng_sample_sorted(g, 10, 10, s) == RCP_OK);
    for (int i = 0; i < 10; ++i) EXPECT(s[i] == i + 1);  // sorted sample of everything
    EXPECT(rcp_rng_sample_sorted(g, 5, 6, s) == RCP_ESEMANTIC);
    rcp_rng_free(g);
    (void)rej;
    double u[3];
    EXPECT(rcp_rng_create(42, RCP_RNG_REJECTION, &g) == RCP_OK);
    EXPECT(rcp_rng_unif(g, 3, u) == RCP_OK);
    EXPECT(u[0] == 0.9148060434963554 && u[1] == 0.9370754132978618 && u[2] == 0.2861395347863436);
    rcp_rng_free(g);
    // big sorted sample through sample.int's hash variant (n > 1e7)
    EXPECT(rcp_rng_create(1, RCP_RNG_REJECTION, &g) == RCP_OK);
    std::vector<int64_t> big(1000);
    EXPECT(rcp_rng_sample_sorted(g, 20000000, 1000, big.data()) == RCP_OK);
    for (int i = 1; i < 1000; ++i) EXPECT(big[i] > big[i - 1] && big[i] <= 20000000);
    rcp_rng_free(g);
    std::printf("abi ok (%d devices)\n", nd);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !std::strcmp(argv[1], "bam")) return bam(argc, argv);
    if (argc >= 2 && !std::strcmp(argv[1], "abi")) return abi();
    std::fprintf(stderr, "usage: abi_driver bam FILE... | abi\n");
    return 2;
}
