// orbfe_common.h — geometry tables shared by the host setup (orbfe_host.hip) and the gfx950 kernels
// (orbfe_kernels.hip).  All tables are computed once per (extractor params, image size) on the host
// with the reference's own float/double arithmetic and uploaded to device memory.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbfe.h"

namespace orbfe {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;          // EDGE_THRESHOLD (ORBextractor.cpp:74)
constexpr int kBorder = kEdge - 3; // minBorderX/Y (ORBextractor.cpp:772-773)
constexpr int kHalfPatch = 15;     // HALF_PATCH_SIZE (:73)
constexpr int kPatchR = 21;        // descriptor patch radius: 18 (max rotated pattern offset) + 3 (blur)
constexpr int kPatchD = 2 * kPatchR + 1;  // 43
// Level coordinates in the FAST slots, the octree's key cache and the level keypoints are packed as
// (x + y * w) | score << 24 with w the level's width: the pixel's row-major index in 24 bits, so every level
// of at most 2^24 pixels (4 096 x 4 096, 4 500 x 2 300, 2 500 x 4 500, ...) fits, whatever its aspect.  Decoding
// divides by w with a per-level magic multiplier (LevelGeo::kmag, ksh; key_xy in the kernels).
constexpr int kKeyXYBits = 24;
constexpr int kMaxCellCoord = 32767;  // CellGeo's int16 ROI coordinates (and its int16 level width)
// compact gather records (k_pack_compact): x | y << 14 | octave << 28, levels up to 16 383 px per side
constexpr int kCompactXYBits = 14;
constexpr int kMaxCellRoi = 64;    // max cell ROI side (wCell+6, hCell+6); checked on the host

// One pyramid level of one image geometry.
struct LevelGeo {
    int w, h;            // level size: cvRound(W * invScale), cvRound(H * invScale) (:1110-1111)
    int pitch;           // row pitch of the level in the pyramid workspace (w rounded up to 16)
    int64_t ws_off;      // byte offset of the level inside an image's pyramid workspace (levels >= 1)
    float scale, inv_scale;
    int n_feat;          // mnFeaturesPerLevel[l]
    int kp_cap;          // capacity of the per-level selected list: max(N+2, 4*nIni) + 2
    int kp_off;          // offset of the level inside an image's level-keypoint array
    float size;          // (float)(int)(PATCH_SIZE * scale) (:836)
    // DistributeOctTree frame (relative to minBorder): [0, maxX-minX) x [0, maxY-minY)
    int span_x, span_y;
    int n_ini;           // round((float)spanX / spanY)
    float hx;            // (float)spanX / nIni
    int cell0, ncell;    // first cell (global cell index) and number of cells of this level
    int key_off;         // offset of the level's dense candidate scratch inside an image
    int key_cap;         // sum of the level's cell slot capacities
    // cv::resize tables (levels >= 1): column table at xtab_off (xofs, a0, a1), row table at ytab_off
    int xtab_off, ytab_off;
    int xmax;            // first column whose sx+1 >= src width
    int xvec;            // end of OpenCV's vectorised span of the vertical pass
    int wide;            // 1: a group's 4th pixel lies past its first 8 source bytes (steps near 2): its taps
                         // come from a window of its own (sx3 - sx0 <= 15; the other pixels' within 8 bytes)
    int area;            // 1: an exact 2x step, cv::resize's INTER_AREA fast path (resizeAreaFast_): the tables
                         // hold the 2x2 average (weights 1024), xvec its vector span, the tail rounds half to even
    // k_resize of this level: groups per row (multiple of 4), most source rows per band, source stride;
    // the launch's dynamic LDS is sized from these (the small levels fit more workgroups per CU)
    int rs_ngrp, rs_nsrc, rs_sp;
    int rs_rows;         // k_resize_rows output rows per band: kRsRows, fewer for a level whose source rows per band
                         // would not fit the LDS (levels wider than ~7 000 px)
    int64_t shear_off;   // byte offset of the level's w x h sheared view inside an image's k_shear output
    // k_octree (bins): every candidate's quadtree path as a Morton code, code = X[x_rel] | Y[y_rel]
    // (host tables at oct_xt / oct_yt of the octree table buffer): column in the bits above 2 * oct_d,
    // then one 2-bit digit per depth 1 .. oct_d (x bit low, y bit high, ExtractorNode::DivideNode's
    // quadrant).  Candidates are counted per depth-oct_d0 node (oct_bins bins, column-major).
    int oct_d, oct_d0, oct_bins;
    int oct_xt, oct_yt, oct_nx, oct_ny;
    // packed level keys (kKeyXYBits): y = mul_hi(xy, kmag) >> ksh, x = xy - y * w for xy < 2^24
    uint32_t kmag;
    int ksh;
};

// One FAST cell (ORBextractor.cpp:788-828): ROI rows [y0,y1), cols [x0,x1) in level coordinates.
struct CellGeo {
    int16_t level, kw;   // kw: the level's width, the radix of its packed keys (k_detect, kKeyXYBits)
    int16_t x0, y0, x1, y1;
    int slot_off;        // offset (in keys) of the cell's output slot inside an image's slot array
    int slot_cap;        // ceil(ww/2)*ceil(wh/2): strict 3x3 NMS keeps at most one pixel per 2x2 block
};

// Resize column entry.
#ifndef ORBFE_RS_ROWS
#define ORBFE_RS_ROWS 16  // experiment switch (tools/dbg/build_variant.sh)
#endif
constexpr int kRsRows = ORBFE_RS_ROWS;  // k_resize output rows per workgroup (band)
// batches of fewer images than this run the small-batch (latency) variants: the one-launch pyramid cascade,
// one FAST cell per wave, 1 024-thread octree workgroups
constexpr int kSmallBatchImages = 32;
// k_octree candidates kept in LDS (with the node arrays <= 80 KiB: two workgroups per CU)
constexpr int kOctKeys = 7424;
// k_octree_bins: keys per block of the first sweep's key -> cell table (log2); a key walks forward from its
// block's first cell over the cells the block spans
#ifndef ORBFE_OB_KBLK_SH
#define ORBFE_OB_KBLK_SH 4  // 16 keys (64: octree 0.421 -> 0.408 ms standalone, 8 pairs 32.9 -> 31.8 us; 8: LDS, 0.574)
#endif
constexpr int kObKblkSh = ORBFE_OB_KBLK_SH;
constexpr int kObKblkMax = 32768 >> kObKblkSh;  // table entries (keys past them walk from the last one)

struct ResizeX {
    int32_t sx;
    int16_t a0, a1;
};
struct ResizeY {
    int32_t sy0, sy1;    // already clipped to [0, src_h)
    int16_t b0, b1;
};

// Per-geometry constants passed by value to every kernel.
struct Geo {
    int nlevels;
    int W, H;
    int ncells;
    int ini_th, min_th;
    int kp_cap;          // per-image capacity of the final keypoint list (sum of level kp_cap)
    int lvl_kp_cap;      // per-image size of the level-keypoint array (same as kp_cap)
    int64_t ws_bytes;    // per-image pyramid workspace bytes (levels >= 1)
    int64_t shear_bytes; // per-image k_shear output (sum of w x h over levels)
    int64_t slot_total;  // per-image cell slot count
    int64_t key_total;   // per-image dense candidate scratch count
    int max_ncap;        // octree node capacity (max over levels of kp_cap)
    int oct_keys;        // octree candidates kept in LDS (kOctKeys, or 0 when the node arrays need the LDS)
    int rs_nsrc;         // k_resize: most source rows one 8-row output band needs
    int rs_sp;           // k_resize: largest source row stride (W for the input, pitch for derived levels)
    int rs_ngrp;         // k_resize: most 4-pixel groups in a derived level row (multiple of 4)
    int max_rh;          // largest FAST cell ROI height (rows)
    int max_rw;          // largest FAST cell ROI width (columns)
    int max_wh;          // largest FAST detection window height (rows)
    int max_win;         // largest FAST detection window (pixels), rounded up to 16
    int fd_mp;           // k_detect: u8 M map pitch in bytes (>= widest window + 6, multiple of 16)
    int fd_pq;           // k_detect: pair-queue entries (>= ceil(ww/2) * wh)
    int fd_alt;          // k_detect: largest cell slot_cap (minTh survivors staged in the ROI area)
    int oct_bins_max;    // k_octree (bins): most bins of any level
    int oct_tab_max;     // k_octree (bins): most X + Y table words of any level
    int oct_kblk_max;    // k_octree (bins): most key blocks of any level (key_cap >> kObKblkSh + 1)
    int oct_v;           // k_octree implementation: 0 bins (default), 1 the per-candidate pass kernel (automatic
                         // when the bins' LDS would exceed 150 KiB, or orbfe_set_octree_kernel)
    int umax[16];
    float scale[kMaxLevels];
    float inv_scale[kMaxLevels];
    LevelGeo lv[kMaxLevels];
};

}  // namespace orbfe
