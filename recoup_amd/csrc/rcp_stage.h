// rcp_stage.h -- host <-> device copies of caller-owned (pageable) host memory through pinned
// staging buffers (rcp_stage.cpp).
//
// The one-shot entry points the R shim binds move the reference's data across PCIe: the reads
// R holds (rcp_readset_create, ~13 B per read) and the R x B double matrix R allocated
// (rcp_profile: 1.6 GB on C4).  HIP copies pageable memory through small internal staging
// buffers at 22-48 GB/s and hipHostRegister of the caller's matrix costs ~70 ms per 1.6 GB
// (profiles/r02/pcie.log); two 64 MB pinned buffers per device, filled / drained by host
// threads while the DMA engine moves the other one, run at 51-54 GB/s (pinned: 55-57).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rcp {

// dst (device) <- src (host); returns once the copy has completed on `stream`.
hipError_t stage_h2d(void* dst, const void* src, size_t bytes, int device, hipStream_t stream);

// dst (host) <- src (device), after everything enqueued on `stream` so far; blocks until done.
// `height` rows of `width` bytes, `spitch` apart on the device and `dpitch` apart on the host --
// e.g. a column-major matrix with a padded device leading dimension, or one GPU's block of rows
// of the caller's R matrix (rows = columns of the matrix).
hipError_t stage_d2h_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                        int device, hipStream_t stream);

// The host -> device copies of the calling thread go through lane `lane` (0 or 1) while this
// object lives: each lane has its own pinned and landing buffers and copy threads, so a second
// thread can upload one array while the first uploads another (rcp_readset_create: chromosome
// codes and strands beside the starts)
class H2dLane {
  public:
    explicit H2dLane(int lane);
    ~H2dLane();
    H2dLane(const H2dLane&) = delete;
    H2dLane& operator=(const H2dLane&) = delete;

  private:
    int prev_;
};

// RCP_TRACE set in the environment: stderr lines per staged copy / pipeline step (diagnostics)
bool trace_on();
double trace_ms();  // a steady clock in ms

// int32 values (read starts) up as 16-bit offsets from per-block minima where the block's span
// allows, strand codes four to a byte (codes outside 0..2 arrive as -1): decoded on the device
// into dst.  Below 2^20 values, or without the device landing buffers: the plain staged copy.
hipError_t stage_h2d_i32(int32_t* dst, const int32_t* src, size_t n, int device, hipStream_t stream);
hipError_t stage_h2d_strand(int8_t* dst, const int8_t* src, size_t n, int device, hipStream_t stream);
// Chromosome codes one byte each when n_codes <= 255 (a code outside [0, n_codes) arrives as -1
// and still drops its read), else as stage_h2d_i32.
hipError_t stage_h2d_codes(int32_t* dst, const int32_t* src, size_t n, int32_t n_codes, int device,
                           hipStream_t stream);
// Read widths end[i] - start[i] + 1 formed on the way and sent packed (a block's widths span far
// less than 2^16 whatever the reads' order, where unsorted ends would go raw) into dst.  *unfit:
// a width outside int32 (nothing usable sent: the caller uploads the ends instead).
hipError_t stage_h2d_width(int32_t* dst, const int32_t* start, const int32_t* end, size_t n, int device,
                           hipStream_t stream, bool* unfit);
// ... and down (Rle runs): blocks packed on the device as their first value + 16-bit offsets,
// expanded by the copy threads; blocks that do not fit are copied as they are
hipError_t stage_d2h_i32(int32_t* dst, const int32_t* src, size_t n, int device, hipStream_t stream);

// A column-major matrix of bin numerators (rows x cols words, column stride sld) into the host's
// double matrix (column stride dld): cell (i, c) = q * scale / div[i] as the device makes a mean
// (rcp_pack_kernel), through the same pinned buffers, expanded by the copy threads.  Waits.
// When the device has no pinned buffers (no stager for its ordinal, hipHostMalloc refused), sets
// *unavailable and returns hipSuccess without copying: the caller downloads the doubles instead.
hipError_t stage_d2h_expand(double* dst, size_t dld, const uint32_t* src, size_t sld, size_t rows, size_t cols,
                            const uint32_t* div, double scale, int device, hipStream_t stream, bool* unavailable);

inline hipError_t stage_d2h(void* dst, const void* src, size_t bytes, int device, hipStream_t stream) {
    return stage_d2h_2d(dst, bytes, src, bytes, bytes, 1, device, stream);
}

}  // namespace rcp
