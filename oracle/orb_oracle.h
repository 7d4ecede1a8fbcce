/*
 * orb_oracle.h — TEST INFRASTRUCTURE ONLY (checker, never shipped, never on the product path).
 *
 * CPU restatement of the reference ORB-SLAM2 extractor (pyORBExtractor/ORBextractor.cpp) and of
 * the OpenCV 4.x primitives it calls.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liborboracle.so.
 *
 * PARITY STATUS: extractor parity is UNPINNED — the reference extractor cannot be built here
 * (it needs OpenCV 4, absent from the image: no headers, libraries or cv2) and the reference
 * holds no extractor output fixtures.  See DESIGN.md §Oracle.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H

#include <stdint.h>

#include "../include/orbfe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full operator_kd (ORBextractor.cpp:1042-1104).  pyr_out (optional) receives the unpadded
 * pyramid levels concatenated level-major (sizes from oracle_level_sizes). */
int oracle_extract(const orbfe_params* p, const uint8_t* img, int32_t w, int32_t h, int32_t stride,
                   orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out, uint8_t* pyr_out);

/* Scale tables + per-level feature counts + umax (ORBextractor.cpp:410-470). */
int oracle_tables(const orbfe_params* p, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                  int32_t* n_per_level, int32_t* umax16);

/* Level sizes (ORBextractor.cpp:1110-1111): wh[2*l] = w_l, wh[2*l+1] = h_l. */
int oracle_level_sizes(const orbfe_params* p, int32_t w, int32_t h, int32_t* wh);

/* cv::resize(INTER_LINEAR) of a u8 image. */
int oracle_resize(const uint8_t* src, int32_t sw, int32_t sh, int32_t sstride, uint8_t* dst, int32_t dw, int32_t dh,
                  int32_t simd_lanes);

/* cv::GaussianBlur(7x7, sigma 2, REFLECT_101) 8U fixed-point path. */
int oracle_blur7(const uint8_t* src, int32_t w, int32_t h, uint8_t* dst);

/* cv::FAST(img, kps, th, nonmax=true) TYPE_9_16 on a w x h ROI.
 * Writes (x, y, score) triples; returns count or ORBFE_ECAPACITY. */
int oracle_fast(const uint8_t* img, int32_t stride, int32_t w, int32_t h, int32_t th, int32_t* xys, int32_t cap);

/* Per-level candidate list (cells + FAST + fallback, ORBextractor.cpp:768-828), in
 * vToDistributeKeys order, coordinates relative to (minBorderX, minBorderY). */
int oracle_level_candidates(const orbfe_params* p, const uint8_t* lvl, int32_t w, int32_t h, int32_t* xyr,
                            int32_t cap);

/* DistributeOctTree (ORBextractor.cpp:539-762) on explicit relative candidates.
 * xyr: n triples (x_rel, y_rel, response); out: selected triples in list order. */
int oracle_octree(const int32_t* xyr, int32_t n, int32_t minX, int32_t maxX, int32_t minY, int32_t maxY,
                  int32_t N, int32_t* out, int32_t cap);

/* SURVEY H1 tie report: per level l, ties[5l] = 1 if the careful phase's `>= N` break
 * (ORBextractor.cpp:729-730) fell inside a run of equal-size nodes (which keypoints the reference keeps
 * depends on heap addresses), ties[5l+1] = runs of >= 2 equal-size nodes the careful phase divided (their
 * keypoints' ORDER depends on addresses), ties[5l+2] = careful-phase iterations, ties[5l+3] / [5l+4] = the
 * straddled run's node count / how many of them were divided. */
int oracle_octree_ties(const orbfe_params* p, const uint8_t* img, int32_t w, int32_t h, int32_t stride, int32_t* ties);

/* cv::fastAtan2. */
float oracle_fast_atan2(float y, float x);

/* glibc 2.35 x86-64 FMA-variant sinf/cosf restated (the reference's (float)cos(float) / sin). */
float oracle_cosf(float x);
float oracle_sinf(float x);

#ifdef __cplusplus
}
#endif

#endif
