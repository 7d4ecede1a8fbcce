// orbfe_kernels.h — launchers of the gfx950 kernels (orbfe_kernels.hip) used by orbfe_host.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "orbfe_common.h"

namespace orbfe {

// Pointers for k_stereo.  Pair p reads left/right data at base + p * stride, which covers both the
// interleaved batch layout (images 2p, 2p+1 of one handle) and two single-image handles (stride 0).
struct StereoArgs {
    const orbfe_keypoint* kpsL;
    const orbfe_keypoint* kpsR;
    int64_t kp_stride;        // keypoints between consecutive pairs (descriptors: kp_stride * 32 bytes)
    const uint8_t* descL;
    const uint8_t* descR;
    const int* countL;
    const int* countR;
    int64_t cnt_stride;
    const uint8_t* lvl0L;     // level 0 = the input images
    const uint8_t* lvl0R;
    int64_t lvl0_stride;
    const uint8_t* wsL;       // levels >= 1
    const uint8_t* wsR;
    int64_t ws_stride;
    float* u_right;
    float* depth;
    int8_t* status;
    int32_t* match_r;
    int64_t out_stride;
    // row buckets (k_stereo_bucket): per pair (H + 1) offsets and bucket_cap right-keypoint indices,
    // plus out_stride compact (x, octave-as-bits) records per pair
    int* bucket_off;
    uint16_t* bucket_idx;
    int64_t bucket_cap;
    float2* rinfo;
    // the right images' level keypoints / counts (octree output) the buckets are built from, and their strides
    // between consecutive pairs
    const uint32_t* lkpR;
    int64_t lkp_stride;
    const int* lcntR;
    int64_t lcnt_stride;
    float maxD;               // np.float32(bf / np.float32(bf / fx32))   (Frame.py:43, 181-183)
    float bf32;               // np.float32(bf): what `mbf / disparity` promotes bf to
    double bf;
};

// k_pack: per-pair fixed-capacity result records (see orbfe_batch_pack_device)
struct PackArgs {
    const int* count;
    const orbfe_keypoint* kps;
    const uint8_t* desc;
    const float* u_right;
    const float* depth;
    const int8_t* status;
    int kp_cap;
    int64_t rec_bytes;
};

hipError_t launch_pack(const PackArgs& a, uint8_t* out, int pair0, int n_pairs, hipStream_t s);
// k_pack_compact: the compact record layout (orbfe_batch_pack_compact_device); inverse level scales by octave
struct CompactScales {
    float inv_scale[kMaxLevels];
};
hipError_t launch_pack_compact(const PackArgs& a, const CompactScales& sc, uint8_t* out, int pair0, int n_pairs,
                               hipStream_t s);
// k_copy_segments: up to 12 dword copies in one launch (dst may be device-visible page-locked host memory)
struct CopySegs {
    struct Seg {
        const uint32_t* src;
        uint32_t* dst;
        uint32_t dwords;
    } seg[12];
    int n;
};
hipError_t launch_copy_segments(const CopySegs& a, hipStream_t s);
// k_undistort: pinhole K (float in the reference: mK is float32) + distortion (k1, k2, p1, p2[, k3])
struct UndistortArgs {
    double fx, fy, cx, cy;
    double k1, k2, p1, p2, k3;
};
hipError_t launch_undistort(const float* xy_in, int n, int stride_in, float* xy_out, const UndistortArgs& a,
                            hipStream_t s);
// zero_word (optional): a device int the launch sets to 0 (the batch's overflow word, cleared without a memset)
hipError_t launch_resize(const Geo& g, int l, const uint8_t* in, int64_t in_pitch, uint8_t* ws, const ResizeX* xt,
                         const ResizeY* yt, int n_images, hipStream_t s, int variant = 0, int* zero_word = nullptr);
hipError_t launch_detect(const Geo& g, const CellGeo* cells, const uint8_t* in, int64_t in_pitch, const uint8_t* ws,
                         int* cell_count, uint32_t* slots, int n_images, hipStream_t s, int variant = 0,
                         int* stats = nullptr);
size_t octree_lds_bytes(const Geo& g, int maxcell);
size_t octree_bins_lds_bytes(const Geo& g, int maxcell);
size_t detect_lds_bytes(const Geo& g);
// k_resize_cascade (all levels in one launch, small batches): strips = n_strips x nlevels x {computed lo, hi,
// owned lo, hi} int16 (host resize_strips); LDS: buffer A at 0, B at off_b, the x selectors at off_x
hipError_t launch_resize_cascade(const Geo& g, const uint8_t* in, int64_t in_pitch, uint8_t* ws, const ResizeX* xt,
                                 const ResizeY* yt, const int16_t* strips, int n_strips, int off_b, int off_x,
                                 int lds_bytes, int n_images, hipStream_t s, int* zero_word = nullptr,
                                 long long* prof = nullptr);
hipError_t prepare_resize_cascade(int lds_bytes);
// raise the octree kernels' dynamic-LDS attribute for this geometry (outside any stream capture)
hipError_t prepare_octree(const Geo& g, int maxcell);
// Geo::oct_v selects k_octree_bins (0) or the per-candidate pass kernel k_octree (1); octab: the
// per-level Morton tables of k_octree_bins (orbfe_host.hip octree_tables)
hipError_t launch_octree(const Geo& g, const CellGeo* cells, const int* cell_count, const uint32_t* slots,
                         const uint32_t* octab, uint32_t* kd, uint16_t* kn, uint32_t* lvl_kp, int* lvl_count, int* overflow,
                         int maxcell, int n_images, hipStream_t s, int variant = 0, long long* prof = nullptr);
// fused IC angle + 7x7 blur of each keypoint's neighbourhood + steered BRIEF (replaces k_blur + k_describe)
// bucket (optional): the stereo row buckets of pairs 0 .. n_bucket - 1 are built by extra workgroups of the
// same launch (they need the octree's level keypoints only); only when orb_fuses_bucket(g)
hipError_t launch_orb(const Geo& g, const uint8_t* in, int64_t in_pitch, const uint8_t* ws, const uint32_t* lvl_kp,
                      const int* lvl_count, orbfe_keypoint* out_kp, uint8_t* out_desc, int* out_count, int n_images,
                      const uint32_t* tab, hipStream_t s, int variant = 0, const StereoArgs* bucket = nullptr,
                      int n_bucket = 0);
bool orb_fuses_bucket(const Geo& g);
// k_orb's item table (orb_tables on the host): 192 horizontal items + 256 centroid slots x 4 dwords
constexpr int kOrbTabWords = 192 + 256 * 4;
// buckets_built: k_orb's launch already built the row buckets (launch_orb's bucket argument)
hipError_t launch_stereo(const Geo& g, const StereoArgs& a, int n_pairs, hipStream_t s, bool buckets_built = false);
// sheared views of every level (GetImagePyramid), out: n_images x g.shear_bytes
hipError_t launch_shear(const Geo& g, const uint8_t* in, int64_t in_pitch, const uint8_t* ws, uint8_t* out, int n_images,
                        hipStream_t s);
hipError_t launch_hamming_matrix(const uint8_t* a, int na, const uint8_t* b, int nb, int* out, hipStream_t s);
hipError_t launch_hamming_search(const uint8_t* q, int nq, const uint8_t* tr, const int* off, const int* idx, int* bd,
                                 int* bi, int* sd, int* si, int* all_d, hipStream_t s);

}  // namespace orbfe
