/*
 * orbfe.h — C-ABI of the MI355X-native ORB front-end (liborbfe.so, gfx950 HIP).
 *
 * Drop-in boundary for the pyOrbSLAM2 front-end hot path.  Each entry point names the reference
 * interface it replaces (paths relative to the reference repo M2219/pyOrbSLAM):
 *
 *   pyORBExtractor.ORBextractor            pyORBExtractor/orb_extractor.cpp:22-38, ORBextractor.h:45-114
 *   Frame.compute_stereo_matches           Frame.py:161-279
 *   ORBMatcher.descriptor_distance / search_by_projection_f_f / _f_p (Hamming core)
 *                                          ORBMatcher.py:12-14, 215-283, 291-393
 *   pyDBoW.TemplatedVocabulary load_from_text_file / transform / transform_feature
 *                                          pyDBoW/TemplatedVocabulary.py:43-81, 108-160
 *
 * Conventions
 *   - plain C types only; caller-owned output buffers; every call returns an int status
 *     (ORBFE_OK = 0, < 0 on error) and the message is kept in a thread-local string
 *     readable with orbfe_last_error();
 *   - one handle per camera / per thread (the reference extractor is stateful and not
 *     re-entrant: ORBextractor.h:88 overwrites mvImagePyramid on every call);
 *   - "device" entry points take device pointers and a hipStream_t passed as void*;
 *     they enqueue work and return without synchronising.
 */
#ifndef ORBFE_H
#define ORBFE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header (orbfe_abi_version() returns the library's).  4: ORBFE_NSTAGES = 5 (stage 3
 * describe, 4 stereo; the round-1 blur stage and orbfe_set_blur_fork are gone), orbfe_set_graphs,
 * orbfe_set_octree_kernel / orbfe_get_octree_kernel, orbfe_debug_detect_stats. */
#define ORBFE_ABI_VERSION 6 /* 6: compact gather records pack x | y << 14 | octave << 28 (was 12 / 12 / 24); level
                               * sides above 4 095 px are accepted (kKeyXYBits) */
/* frames whose sheared pyramids the lazy frame path (want_pyramid = 2) keeps on the device */
#define ORBFE_FRAME_RING 8
int32_t orbfe_abi_version(void);

#define ORBFE_OK 0
#define ORBFE_EINVAL (-1)    /* bad argument / unsupported configuration            */
#define ORBFE_ENOMEM (-2)    /* host or device allocation failed                    */
#define ORBFE_EHIP (-3)      /* HIP runtime error (message from hipGetErrorString)   */
#define ORBFE_ECAPACITY (-4) /* caller buffer too small (*n_out holds the need)     */
#define ORBFE_ESTATE (-5)    /* call order violated (e.g. pyramid before extract)   */
#define ORBFE_EOVERFLOW (-6) /* an on-device capacity bound was exceeded            */
#define ORBFE_EFORMAT (-7)   /* malformed input file (vocabulary text)              */
#define ORBFE_EREJECT (-8)   /* vocabulary header outside the accepted ranges       */

/* ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
 * (orb_extractor.cpp:23; ORBextractor.cpp:410-470). */
typedef struct orbfe_params {
    int32_t nfeatures;
    float scale_factor; /* narrowed to float exactly like the pybind11 float argument */
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    /* Lane count of OpenCV's vectorised vertical resize pass (cv::resize INTER_LINEAR 8U,
     * SURVEY.md Appendix A.2 / H2): 16 = CV_SIMD128 baseline build (default), 32 = AVX2-wide
     * build, 0 = scalar formula everywhere.  OpenCV is not vendored by the reference; this is
     * the only unpinned knob of the pixel arithmetic. */
    int32_t resize_simd_lanes;
} orbfe_params;

/* cv::KeyPoint as the reference's caster returns it: (pt.x, pt.y, size, angle, response,
 * octave) (opencv_type_casters.h:106-108).  24 bytes, naturally aligned. */
typedef struct orbfe_keypoint {
    float x, y, size, angle, response;
    int32_t octave;
} orbfe_keypoint;

typedef struct orbfe_ctx* orbfe_handle;

/* ---- lifetime ------------------------------------------------------------------------ */

/* ORBextractor::ORBextractor (ORBextractor.cpp:410-470). */
int orbfe_create(const orbfe_params* params, orbfe_handle* out);
int orbfe_destroy(orbfe_handle h);
const char* orbfe_last_error(void);
/* library build string ("gfx950 ...") */
const char* orbfe_version(void);

/* Build identity: the first 16 hex digits of the SHA-256 of the sources and headers the library was built
 * from (Makefile).  Measurement files (profiles/traffic.json, profiles/valu.json) record it, and bench.py
 * uses their per-kernel figures only when it matches the loaded library. */
const char* orbfe_build_id(void);

/* GetLevels/GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/
 * GetInverseScaleSigmaSquares (ORBextractor.h:62-82).  Each array has nlevels floats; any
 * pointer may be NULL.  n_per_level receives mnFeaturesPerLevel (ORBextractor.cpp:435-446). */
int orbfe_get_scales(orbfe_handle h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                     int32_t* n_per_level);

/* ---- host-buffer drop-in (one image per call) ------------------------------------------ */

/* ORBextractor::operator_kd (ORBextractor.cpp:1042-1104) as bound at orb_extractor.cpp:31-38.
 * img: width x height u8, row stride `stride` bytes (the reference ignores numpy strides and
 * requires C-contiguous input; pass stride = width for identical behaviour).
 * Writes up to `cap` keypoints and cap*32 descriptor bytes; *n_out = number produced.
 * An empty image (width or height 0) yields *n_out = 0 (ORBextractor.cpp:1045-1046). */
int orbfe_extract(orbfe_handle h, const uint8_t* img, int32_t width, int32_t height, int32_t stride,
                  orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out);

/* GetImagePyramid (orb_extractor.cpp:30): pyramid level `level` of the last orbfe_extract.
 * sheared = 1 reproduces the reference's Mat->ndarray caster, which ignores Mat::step and so
 * returns row r of a level as bytes [19*(w+38)+19 + r*w, ... + w) of the 19-px reflect-101
 * padded buffer (opencv_type_casters.h:232-239; ORBextractor.cpp:1112-1128);
 * sheared = 0 returns the true w x h level.  out must hold w*h bytes (sizes via w_out, h_out;
 * call with out = NULL to query the size). */
int orbfe_pyramid(orbfe_handle h, int32_t level, uint8_t* out, int32_t sheared, int32_t* w_out,
                  int32_t* h_out);

/* Frame.compute_stereo_matches (Frame.py:161-279) on the last left/right extraction of two
 * handles (left = hl, right = hr; both must have extracted same-size images).
 * bf = Frame.mbf (Python float), fx = Frame.mK[0][0] (np.float32).
 * Outputs, each of length nL = number of left keypoints:
 *   status[i] = 0  no match      (reference keeps Python int -1)
 *             = 1  matched       (reference stores np.float32 uR / depth: u_right / depth)
 *             = 2  zero disparity: the reference substitutes disparity = 0.01 in Python double
 *                  precision (Frame.py:273-275); u_right/depth then hold uL-0.01 and bf/0.01
 *                  rounded to f32 and the host layer recomputes them in double.
 *   match_r[i] = index of the right keypoint chosen by the Hamming search (or -1). */
int orbfe_stereo_match(orbfe_handle hl, orbfe_handle hr, double bf, float fx, float* u_right, float* depth,
                       int8_t* status, int32_t* match_r, int32_t n_left);

/* ---- per-frame stereo path (one Frame, one enqueue) ------------------------------------------
 * Frame.__init__ (Frame.py:48-65) calls ExtractORB(0, left), ExtractORB(1, right) — two synchronous
 * operator_kd calls, ORBextractor.cpp:1042-1104 — then GetImagePyramid on both extractors
 * (orb_extractor.cpp:30) and compute_stereo_matches (Frame.py:161-279).  orbfe_frame_extract does all
 * of it for one stereo pair in ONE enqueue on the handle's stream: both images copied in, the 2-image
 * pipeline, the stereo match, optionally the sheared pyramids of both images (built on the device), and
 * every result copied into page-locked host memory before a single synchronisation.  The fetch calls
 * below then only copy host memory.  Both images are width x height u8 with row stride `stride`; an
 * empty image (width or height 0) yields no keypoints (ORBextractor.cpp:1045-1046).  bf / fx as in
 * orbfe_stereo_match.  want_pyramid: 0 none (orbfe_frame_pyramid builds them on request), 1 the sheared
 * views copied into the frame buffer with the results, 2 lazy: the views stay in a device ring of
 * ORBFE_FRAME_RING frames and cross PCIe only when orbfe_frame_pyramid_fetch asks for them (Frame.py:59-60
 * keeps the lists, but the tracking loop rarely reads them). */
int orbfe_frame_extract(orbfe_handle h, const uint8_t* left, const uint8_t* right, int32_t width, int32_t height,
                        int32_t stride, double bf, float fx, int32_t want_pyramid);
/* keypoints / descriptors of side 0 (left) or 1 (right) of the last frame (operator_kd's outputs) */
int orbfe_frame_fetch(orbfe_handle h, int32_t side, orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out);
/* stereo results of the last frame (layout and meaning as orbfe_stereo_match; *n_out = left count) */
int orbfe_frame_fetch_stereo(orbfe_handle h, float* u_right, float* depth, int8_t* status, int32_t* match_r,
                             int32_t cap, int32_t* n_out);
/* GetImagePyramid()[level] of side 0 / 1 of the last frame: the reference's sheared view (see
 * orbfe_pyramid).  Built at extraction when want_pyramid was set, otherwise now.  out = NULL queries
 * the size. */
int orbfe_frame_pyramid(orbfe_handle h, int32_t side, int32_t level, uint8_t* out, int32_t* w_out, int32_t* h_out);
/* serial number of the last frame (1, 2, ...) and the oldest serial the ring can still hold (a frame extracted
 * with want_pyramid != 2, or before a geometry change, is not in it) */
int orbfe_frame_serial(orbfe_handle h, int64_t* serial, int64_t* oldest);
/* both sheared pyramids' bytes of side 0 / 1 of frame `serial` (extracted with want_pyramid = 2): every
 * level's w_l x h_l view at its shear offset (levels concatenated, 4-byte aligned; bytes = the geometry's
 * shear size, orbfe_batch_view_get).  ORBFE_ESTATE once ORBFE_FRAME_RING newer frames have replaced it. */
int orbfe_frame_pyramid_fetch(orbfe_handle h, int64_t serial, int32_t side, uint8_t* out, int64_t bytes);

/* cv::undistortPoints(pts, K, D, noArray(), K) as Frame.undistort_keypoints (Frame.py:306) and
 * Tracking.compute_image_bounds (Tracking.py:132) call it: OpenCV 4.x's 5-iteration fixed point in double
 * (k_undistort).  K4 = (fx, fy, cx, cy) and dist = (k1, k2, p1, p2[, k3]) as float (the reference keeps
 * mK and mDistCoef in float32); xy: n points at `stride` floats apart (x, y first); out: n x 2 floats.
 * Parity is unpinned: OpenCV is absent and the reference's distorted branch is unreachable (NameError
 * on `mvKeys` at Frame.py:299); DESIGN.md §2 states the semantics followed. */
int orbfe_undistort_points(orbfe_handle h, const float* K4, const float* dist, int32_t n_dist, const float* xy, int32_t n,
                           int32_t stride, float* out);

/* ---- device batch API (bench / batched-frames mode) ----------------------------------------
 * Images are device-resident, n_images x (height x img_pitch) u8, stereo pair p = images
 * (2p, 2p+1) = (left, right).  Results stay on device in handle-owned buffers. */

/* Allocate device workspace for up to max_images images of width x height (idempotent for the
 * same geometry). */
int orbfe_batch_reserve(orbfe_handle h, int32_t width, int32_t height, int32_t max_images);

/* Run the whole extractor on n_images device images (no host synchronisation). */
int orbfe_extract_batch_device(orbfe_handle h, const uint8_t* d_images, int64_t img_pitch, int32_t n_images,
                               void* hip_stream);

/* Stereo-match n_pairs pairs of the last batch extraction (images 2p, 2p+1). */
int orbfe_stereo_batch_device(orbfe_handle h, int32_t n_pairs, double bf, float fx, void* hip_stream);

/* Convenience: extract + stereo for n_pairs pairs in one enqueue (the benchmark step). */
int orbfe_frontend_batch_device(orbfe_handle h, const uint8_t* d_images, int64_t img_pitch, int32_t n_pairs,
                                double bf, float fx, void* hip_stream);

/* orbfe_set_lanes: orbfe_frontend_batch_device runs its batch as min(lanes, n_pairs) contiguous chunks,
 * each on an internal stream (fork from / join into the caller's stream); 1..4, default 4.  Results and
 * their layout do not depend on it. */
int orbfe_set_lanes(orbfe_handle h, int32_t lanes);

/* orbfe_set_graphs(mask): which enqueues run as a HIP graph, captured on the first call with a given
 * (buffers, pointers, sizes, bf, fx) key and replayed with one hipGraphLaunch afterwards (up to 8 cached
 * graphs per handle, dropped when the handle's buffers are reallocated): ORBFE_GRAPH_FRAME =
 * orbfe_frame_extract (default: the per-frame path runs on one stream, a graph saves its launches),
 * ORBFE_GRAPH_BATCH = orbfe_frontend_batch_device with one lane (off by default: graph launches of handles on
 * different streams measured to serialise their chains, 0.27 -> 0.40 ms for 8 pairs as 4 handles).  0 =
 * every operation launched on the stream.  Results do not depend on it; profiling (orbfe_profile_begin)
 * always takes the stream path.  orbfe_graph_stats: captures and graph launches so far, graphs cached now
 * (any pointer may be NULL). */
#define ORBFE_GRAPH_FRAME 1
#define ORBFE_GRAPH_BATCH 2
int orbfe_set_graphs(orbfe_handle h, int32_t mask);
int orbfe_graph_stats(orbfe_handle h, int64_t* captures, int64_t* launches, int32_t* cached);

/* Device result layout of the last batch (pointers into handle-owned device memory):
 *   kps   : n_images x cap  orbfe_keypoint   (cap = *kp_cap)
 *   desc  : n_images x cap x 32 u8
 *   count : n_images int32
 *   u_right, depth : n_pairs x cap float; status : n_pairs x cap int8; match_r : n_pairs x cap int32 */
typedef struct orbfe_batch_view {
    int32_t kp_cap;
    int32_t n_images;
    int32_t n_pairs;
    orbfe_keypoint* kps;
    uint8_t* desc;
    int32_t* count;
    float* u_right;
    float* depth;
    int8_t* status;
    int32_t* match_r;
    int32_t* overflow; /* device int: non-zero if a capacity bound was hit in the last batch */
} orbfe_batch_view;
int orbfe_batch_view_get(orbfe_handle h, orbfe_batch_view* view);

/* Synchronise the handle's last stream and read the overflow word of the last batch (0 = every
 * on-device capacity bound held; otherwise the OR of the codes of the bounds that were hit). */
int orbfe_batch_status(orbfe_handle h, int32_t* overflow);

/* Batched-frames mode, multi-GPU: every pair's results as one fixed-capacity byte record, packed on the
 * device for the rank-0 gather (north star: "RCCL over xGMI only for the trivial gather of per-frame
 * keypoints").  Record layout (pyorbslam_amd/dist.py): counts L, R (2 x i32) | keypoints L, R
 * (kp_cap x orbfe_keypoint each) | descriptors L, R (kp_cap x 32 B each) | u_right, depth (kp_cap x f32)
 * | status (kp_cap x i8), padded to 16 bytes: orbfe_batch_record_bytes.  orbfe_batch_pack_device writes
 * pairs [pair0, pair0 + n_pairs) of the last stereo batch to d_records (n_pairs x rec_bytes, 4-byte
 * aligned) on hip_stream, without synchronising.  d_records is device memory or page-locked host memory
 * (hipHostMalloc): the records then go over PCIe straight into host memory (no device staging buffer, no
 * copy-engine transfer); pageable memory is refused with ORBFE_EINVAL.
 * Ordering (both pack calls): on the batch's own stream the pack simply follows it.  On another stream the
 * pack waits on an event recorded on the batch's stream WHEN THE PACK IS CALLED, so (a) that stream must
 * still exist and must not be inside a graph capture at that moment, and (b) whatever was queued on it after
 * the batch and before the pack call is waited for too. */
int orbfe_batch_record_bytes(orbfe_handle h, int64_t* bytes);
/* Compact records (the host-fed D2H leg and the rank-0 gather, 25 % smaller): counts L, R (2 x i32) |
 * keypoints L, R (kp_cap x {u32 x | y << 14 | octave << 28 in the keypoint's level pixels, f32 angle}) |
 * descriptors L, R (kp_cap x 32 B) | u_right, depth (kp_cap x f32) | FAST scores L, R (kp_cap x u8) | status
 * (kp_cap x i8), padded to 16 bytes (8 + 91 kp_cap).  The keypoint tuples follow exactly: x = f32(level x) *
 * scale[octave] (ORBextractor.cpp:1094-1099), size = (float)(int)(31 * scale[octave]), response = score
 * (pyorbslam_amd.dist.unpack_compact).  Device memory only. */
int orbfe_batch_compact_record_bytes(orbfe_handle h, int64_t* bytes);
int orbfe_batch_pack_compact_device(orbfe_handle h, uint8_t* d_records, int64_t rec_bytes, int32_t pair0,
                                    int32_t n_pairs, void* hip_stream);
int orbfe_batch_pack_device(orbfe_handle h, uint8_t* d_records, int64_t rec_bytes, int32_t pair0, int32_t n_pairs,
                            void* hip_stream);

/* Copy the results of image `image` (and of pair image/2 when image is even and a stereo
 * batch ran) of the last batch to host buffers.  Synchronises the handle's last stream. */
int orbfe_batch_fetch(orbfe_handle h, int32_t image, orbfe_keypoint* kps, uint8_t* desc, int32_t cap,
                      int32_t* n_out);

/* Copy the stereo results of pair `pair` of the last batch (see orbfe_stereo_match for the meaning
 * of the arrays; *n_out = left keypoint count of the pair).  Synchronises the last stream. */
int orbfe_batch_fetch_stereo(orbfe_handle h, int32_t pair, float* u_right, float* depth, int8_t* status,
                             int32_t* match_r, int32_t cap, int32_t* n_out);

/* ---- Hamming search (ORBMatcher core) -------------------------------------------------------
 * ORBMatcher.descriptor_distance (ORBMatcher.py:12-14): popcount(a ^ b) over 32 bytes, batched.
 * For query q the candidates are cand_idx[cand_off[q] .. cand_off[q+1]) (indices into
 * train_desc), scanned in order; the search keeps the FIRST strict minimum (best) and the
 * second-best distance with its candidate exactly as search_by_projection_f_p does
 * (ORBMatcher.py:252-274: `dist < best` shifts best into second; `elif dist < best2`).
 * Distances start at 256 (no candidate => best_idx = -1).  Host pointers; n_query may be 0. */
int orbfe_hamming_search(orbfe_handle h, const uint8_t* query_desc, int32_t n_query, const uint8_t* train_desc,
                         int32_t n_train, const int32_t* cand_off, const int32_t* cand_idx, int32_t* best_dist,
                         int32_t* best_idx, int32_t* second_dist, int32_t* second_idx);

/* Every candidate distance, in CSR order: out_dist[k] = popcount(query[q] ^ train[cand_idx[k]]) for
 * k in [cand_off[q], cand_off[q+1]).  Used by the ORBMatcher drop-in, whose control flow (already
 * matched points, stereo gate, best/second bookkeeping) depends on matches made earlier in the
 * same search and therefore stays sequential on the host. */
int orbfe_hamming_csr(orbfe_handle h, const uint8_t* query_desc, int32_t n_query, const uint8_t* train_desc,
                      int32_t n_train, const int32_t* cand_off, const int32_t* cand_idx, int32_t* out_dist);

/* ORBMatcher.descriptor_distance for ONE pair (ORBMatcher.py:12-14; Frame.py:324-326; MapPoint.py:76-78):
 * popcount(a ^ b) over 32 bytes, computed on the host (a device round trip costs more than the
 * reference's ~10 us Python call; batches go through the kernels above / below). */
int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b, int32_t* out);

/* Frame.get_features_in_area (Frame.py:373-416) for n_q queries at once, on the host: the frame's 64 x 48
 * grid (Frame.assign_features_to_grid, Frame.py:152-159) as CSR (cell (ix, iy) = cell_off[ix * rows + iy]
 * .. cell_off[ix * rows + iy + 1) into cell_idx, the reference's list order), the keypoints' pt (double
 * values of the Python floats) and octave, frame4 = (mnMinX, mnMinY, mfGridElementWidthInv,
 * mfGridElementHeightInv); query q = (x, y, r, min_level, max_level) in double.  Candidates of query q:
 * out_idx[out_off[q] .. out_off[q + 1]), in the reference's order.  ORBFE_ECAPACITY if more than cap
 * (out_off[n_q] then holds the total).  The ORBMatcher drop-in uses it when every operand is a double. */
int orbfe_grid_query(const int32_t* cell_off, const int32_t* cell_idx, int32_t cols, int32_t rows, const double* kp_x,
                     const double* kp_y, const int32_t* kp_oct, int32_t n_kp, const double* frame4, int32_t n_q,
                     const double* qx, const double* qy, const double* qr, const int32_t* qmin, const int32_t* qmax,
                     int32_t* out_off, int32_t* out_idx, int64_t cap);

/* The sequential candidate selection of the tracking searches over precomputed distances (host code), for
 * the ORBMatcher drop-in's double-typed fast path.  Queries are taken in order; query q's candidates are
 * idx[off[q] .. off[q + 1]) with Hamming distances dist[...] (orbfe_hamming_csr); u_right = the frame's
 * mvuRight as doubles (-1 for none); blocked[i] = 1 when frame slot i holds a map point with observations,
 * updated in place with q_obs[q] when query q's map point takes slot best_idx[q] (-1: no match).
 * orbfe_select_f_f: search_by_projection_f_f's inner loop and TH_HIGH test (ORBMatcher.py:348-372): stereo
 * gate |(u - mbf * invzc) - uR| > radius in double.  orbfe_select_f_p: search_by_projection_f_p's
 * (ORBMatcher.py:246-281): gate |xr - uR| > r_scaled, best / second best with their keypoint octaves and
 * the ratio test best > nnratio * second when both are on one octave. */
int orbfe_select_f_f(int32_t n_q, const int32_t* off, const int32_t* idx, const int32_t* dist, const double* u,
                     const double* invzc, const double* radius, const uint8_t* q_obs, const double* u_right,
                     uint8_t* blocked, int32_t n_frame, double mbf, int32_t th_high, int32_t* best_idx);
int orbfe_select_f_p(int32_t n_q, const int32_t* off, const int32_t* idx, const int32_t* dist, const double* xr,
                     const double* r_scaled, const int32_t* kp_octave, const uint8_t* q_obs, const double* u_right,
                     uint8_t* blocked, int32_t n_frame, double nnratio, int32_t th_high, int32_t* best_idx);

/* All-pairs Hamming distance matrix (n_a x n_b int32) — descriptor_distance batched. */
int orbfe_hamming_matrix(orbfe_handle h, const uint8_t* a_desc, int32_t n_a, const uint8_t* b_desc, int32_t n_b,
                         int32_t* out);

/* ---- image ingest (stereo_kitti.py:42-43: cv2.imread(path, cv2.IMREAD_GRAYSCALE)) ------------------
 * PNG (8-bit grey / RGB / grey+alpha / RGBA, non-interlaced) to 8-bit grey, decoded natively (zlib inflate
 * + row unfiltering; colour converted with libpng's rgb_to_gray fixed-point weights as OpenCV requests).
 * orbfe_png_decode: one image from memory; out = NULL returns the size only; `stride` bytes per out row.
 * orbfe_png_read_batch: n files of one size decoded by `threads` host threads into out (n x h x w,
 * contiguous), e.g. pinned staging for one host-to-device copy of a batch of stereo pairs. */
int orbfe_png_decode(const uint8_t* data, int64_t size, uint8_t* out, int64_t stride, int32_t* width, int32_t* height);
int orbfe_png_read_batch(const char* const* paths, int32_t n, int32_t width, int32_t height, uint8_t* out,
                         int32_t threads);

/* ---- live stage timing --------------------------------------------------------------------------
 * While profiling is on, every batch enqueued on the handle records HIP events around its stages:
 * 0 resize (all pyramid levels), 1 detect (FAST cells), 2 octree, 3 describe (k_orb: IC angle +
 * per-keypoint 7x7 blur + steered BRIEF), 4 stereo (row buckets + k_stereo).
 * orbfe_profile_read synchronises and returns the summed milliseconds per stage (ms_per_stage holds
 * ORBFE_NSTAGES floats) over the recorded batches. */
#define ORBFE_NSTAGES 5
int orbfe_profile_begin(orbfe_handle h, int32_t max_batches);
int orbfe_profile_read(orbfe_handle h, float* ms_per_stage, int32_t* n_batches);

/* Kernel micro-benchmark on the inputs of the last batch (development aid, not part of the drop-in):
 * runs stage `stage` (0 resize, 1 detect, 2 octree, 3 describe, 4 stereo) in ablation variant `variant`
 * (0 = production kernel) `reps` times on the handle's last stream and returns the average ms.
 * Variants other than 0 overwrite stage outputs with garbage: re-run the batch afterwards. */
int orbfe_microbench(orbfe_handle h, int32_t stage, int32_t variant, int32_t reps, float* ms);

/* ---- diagnostics (stage outputs of the last orbfe_extract, image 0) ------------------------------
 * orbfe_debug_candidates: the level's FAST cell output in vToDistributeKeys order
 *   (ORBextractor.cpp:808-824), as (x_rel, y_rel, score) triples relative to (minBorderX, minBorderY).
 * orbfe_debug_selected: DistributeOctTree's result for the level in list order
 *   (ORBextractor.cpp:833-834), as (x_rel, y_rel, score) triples. */
int orbfe_debug_candidates(orbfe_handle h, int32_t level, int32_t* xyr, int32_t cap, int32_t* n_out);
int orbfe_debug_selected(orbfe_handle h, int32_t level, int32_t* xyr, int32_t cap, int32_t* n_out);
/* orbfe_debug_octree_profile: re-runs the last batch's octree stage with wall-clock marks (100 MHz ticks,
 * 64 per (image, level), 0 = not reached) written by each workgroup's first thread; development aid. */
int orbfe_debug_octree_profile(orbfe_handle h, int64_t* marks, int64_t n);
/* orbfe_debug_cascade_profile: re-runs the last batch's one-launch pyramid (k_resize_cascade; batches below 32
 * images) with wall-clock marks, 32 per (image, strip) (0 start, 1 level-0 rows staged, 2 + l level l begins,
 * 12 + l level l done); *n_strips = the strip count; development aid. */
int orbfe_debug_cascade_profile(orbfe_handle h, int64_t* marks, int64_t n_marks, int32_t* n_strips);
/* orbfe_debug_detect_stats: re-runs the last batch's FAST cell stage (idempotent) with counters:
 * stats[0] = cells processed, stats[1] = cells whose iniTh / minTh queues met so that the cell took the
 * one-pass path (both thresholds over the minTh queue), stats[2] = cells that fell back to minTh
 * (ORBextractor.cpp:811-815) on the two-queue path.  Development aid; results are unchanged. */
int orbfe_debug_detect_stats(orbfe_handle h, int64_t* stats);

/* DistributeOctTree implementation (ORBextractor.cpp:539-762; results are identical): 0 = automatic
 * (k_octree_bins, or the per-candidate k_octree when the bins' LDS carve would exceed 150 KiB), 1 = always
 * the per-candidate k_octree.  orbfe_get_octree_kernel reports the reserved geometry's choice (0 bins,
 * 1 per-candidate) and the bins kernel's LDS need. */
int orbfe_set_octree_kernel(orbfe_handle h, int32_t kernel);
int orbfe_get_octree_kernel(orbfe_handle h, int32_t* kernel, int64_t* bins_lds_bytes);

/* ---- bag-of-words vocabulary (pyDBoW/TemplatedVocabulary.py) ---------------------------
 *
 * A vocabulary tree of ORB descriptors.  Node 0 is the root; every other node has a parent with a
 * smaller id, and a node's children are ordered by id (the order TemplatedVocabulary.py:62-79 appends
 * them).  A node is a leaf when it has no children (Node.is_leaf, TemplatedVocabulary.py:19-20);
 * word ids number the nodes FLAGGED as leaves in id order (other nodes report word 0).  Parsing and
 * the node tables live on the host; the device copy is made on the first transform. */
typedef struct orbfe_vocab* orbfe_vocab_handle;

typedef struct orbfe_vocab_info {
    int32_t k, L;              /* header branching factor and depth (TemplatedVocabulary.py:46-47) */
    int32_t scoring, weighting; /* header codes n1, n2 (TemplatedVocabulary.py:48-49, 55-56)     */
    int64_t n_nodes;           /* including the root                                            */
    int64_t n_words;           /* flagged leaves: TemplatedVocabulary.size()                    */
    int32_t depth;             /* longest root-to-leaf path                                     */
    int32_t max_children;
} orbfe_vocab_info;

/* TemplatedVocabulary.load_from_text_file (TemplatedVocabulary.py:43-81), parsed natively.
 * Header "k L n1 n2"; ORBFE_EREJECT when 0<=k<=20, 1<=L<=10, 0<=n1<=5, 0<=n2<=3 fails (the
 * reference prints a message and returns False).  Each following line: parent is_leaf d0..d31
 * weight, with byte values in [0,255] and parent < node id; anything else is ORBFE_EFORMAT. */
int orbfe_vocab_load_text(const char* path, orbfe_vocab_handle* out);
/* The same tree from arrays: n_nodes entries each (entry 0 = root, its parent/desc ignored). */
int orbfe_vocab_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int64_t n_nodes,
                       const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc32, const double* weight,
                       orbfe_vocab_handle* out);
int orbfe_vocab_destroy(orbfe_vocab_handle v);
int orbfe_vocab_get_info(orbfe_vocab_handle v, orbfe_vocab_info* info);
/* Host copies of the node tables (any pointer may be NULL); n_nodes entries each. */
int orbfe_vocab_get_nodes(orbfe_vocab_handle v, int32_t* parent, uint8_t* is_leaf, uint8_t* desc32, double* weight,
                          int32_t* word_id);

/* Descent of n descriptors (TemplatedVocabulary.transform_feature, TemplatedVocabulary.py:131-160):
 * from the root, move to the child at the smallest Hamming distance (first child on ties) until a
 * node without children.  word_id / weight are that node's; node_id is the node entered at depth
 * nid_level, or -1 when the descent stopped above it (the reference then keeps the previous
 * feature's value, which the caller threads; TemplatedVocabulary.py:118-123).  Host buffers,
 * synchronous. */
int orbfe_vocab_transform(orbfe_vocab_handle v, const uint8_t* desc32, int64_t n, int32_t nid_level,
                          int32_t* word_id, int32_t* node_id, double* weight);
/* Same on device pointers, enqueued on hip_stream (void* = hipStream_t) without synchronising. */
int orbfe_vocab_transform_device(orbfe_vocab_handle v, const uint8_t* d_desc32, int64_t n, int32_t nid_level,
                                 int32_t* d_word_id, int32_t* d_node_id, double* d_weight, void* hip_stream);
/* Kernel time of the last orbfe_vocab_transform (ms, HIP events), for measurement. */
int orbfe_vocab_last_ms(orbfe_vocab_handle v, float* ms);

#ifdef __cplusplus
}
#endif

#endif /* ORBFE_H */
