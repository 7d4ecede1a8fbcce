// orbfe_host.hip — C-ABI (include/orbfe.h) of the gfx950 ORB front-end: extractor handle, geometry
// tables, device workspace and the enqueue of the kernel pipeline.
//
// Host arithmetic that feeds the kernels (scale tables, level sizes, cell grid, resize coefficients) is
// computed here with the same float/double expressions as the reference (ORBextractor.cpp:410-470,
// 764-828, 1106-1132; OpenCV resize coefficient setup), so every kernel consumes identical integers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbfe_common.h"
#include "orbfe_host_util.h"
#include "orbfe_kernels.h"

using namespace orbfe;

namespace orbfe {
thread_local std::string g_err;
}

namespace {

inline int round_even_f(float v) { return (int)std::lrintf(v); }
inline int floor_f(float v) { int i = (int)v; return i - (i > v); }
inline int ceil_f(float v) { int i = (int)v; return i + (i < v); }
inline short sat_short(int v) { return (short)std::min(std::max(v, -32768), 32767); }

}  // namespace

// concurrent chunks of orbfe_frontend_batch_device (the box exposes 4 hardware queues per process)
constexpr int kLanes = 4;
// frames whose sheared pyramids the lazy frame path keeps on the device (include/orbfe.h ORBFE_FRAME_RING)
constexpr int kFrameRing = ORBFE_FRAME_RING;
// profiling events per batch: stage k (resize, detect, octree, describe, stereo) spans events k -> k + 1;
// see prof_mark
constexpr int kProfEvents = ORBFE_NSTAGES + 1;

struct orbfe_ctx {
    orbfe_params prm{};
    double scale_factor_d = 1.2;
    std::vector<float> sf, isf, s2, is2;
    std::vector<int> n_per_level;
    int umax[16] = {0};

    // geometry of the reserved image size
    int W = 0, H = 0, max_images = 0;
    Geo geo{};
    std::vector<CellGeo> cells;
    std::vector<ResizeX> xt;
    std::vector<ResizeY> yt;
    std::vector<uint32_t> octab;  // k_octree (bins): per-level Morton tables X / Y (octree_tables)
    int maxcell = 0;

    DevBuf<CellGeo> d_cells;
    DevBuf<ResizeX> d_xt;
    DevBuf<uint32_t> d_orb; // k_orb: horizontal items of the sample disc + centroid slots (orb_tables)
    DevBuf<ResizeY> d_yt;
    DevBuf<uint32_t> d_octab;
    DevBuf<uint8_t> d_in;      // staging of the host-buffer API
    DevBuf<uint8_t> d_ws;
    DevBuf<int> d_cell_count;
    DevBuf<uint32_t> d_slots;
    DevBuf<uint32_t> d_kd;
    DevBuf<uint16_t> d_kn;
    DevBuf<uint32_t> d_lvl_kp;
    DevBuf<int> d_lvl_count;
    DevBuf<orbfe_keypoint> d_kps;
    DevBuf<uint8_t> d_desc;
    DevBuf<int> d_count;
    DevBuf<int> d_overflow;
    DevBuf<float> d_uR, d_depth;
    DevBuf<int8_t> d_status;
    DevBuf<int32_t> d_match;
    DevBuf<int> d_boff;
    DevBuf<uint16_t> d_bidx;
    DevBuf<float2> d_rinfo;
    int64_t bucket_cap = 0;
    // hamming scratch, shared by the orbfe_hamming_* calls on this handle; they may come from several
    // threads (the reference runs Tracking, LocalMapping and LoopClosing as threads that all call
    // ORBMatcher / MapPoint, System.py:59-64), so those calls hold hmu for their whole duration
    DevBuf<uint8_t> d_hq, d_ht;
    DevBuf<int> d_hoff, d_hidx, d_hres;
    std::mutex hmu;

    // live profiling: kProfEvents events per batch (see prof_mark)
    std::vector<hipEvent_t> prof_ev;
    int prof_max = 0, prof_n = 0;
    bool prof_on = false;

    hipStream_t own_stream = nullptr;
    bool octree_force = false;  // orbfe_set_octree_kernel(h, 1): the per-candidate k_octree at every geometry
    // k_resize_cascade strip tables of the reserved geometry, per strip count (resize_strips)
    struct Cascade {
        int S = 0, off_b = 0, off_x = 0, lds = 0;
        DevBuf<int16_t> tab;
    };
    std::vector<std::unique_ptr<Cascade>> cascades;
    int cascade_force = 0;  // orbfe_microbench: 0 automatic, > 0 that strip count, -1 never
    // HIP graphs (orbfe_set_graphs, default on): a batch's or a frame's whole enqueue is captured once per
    // (buffers, arguments) key into an executable graph and replayed with one hipGraphLaunch.  gen counts the
    // reallocations of the handle's buffers / geometry changes, which every key includes; a capture goes on
    // cap_stream, so the caller's stream only ever sees the launches.
    int graph_mask = ORBFE_GRAPH_FRAME;  // orbfe_set_graphs: which enqueues replay graphs
    uint64_t gen = 0;
    hipStream_t cap_stream = nullptr;
    struct GraphEntry {
        std::vector<uint64_t> key;
        hipGraphExec_t exec;
        hipEvent_t done;  // recorded after every launch of exec: retire() waits for it before destroying
    };
    std::vector<GraphEntry> graphs;
    int64_t graph_launches = 0, graph_captures = 0;
    // orbfe_frontend_batch_device: up to kLanes concurrent chunks of the batch on internal streams
    int lanes = kLanes;  // orbfe_set_lanes
    hipStream_t lane_stream[kLanes] = {};
    hipEvent_t lane_done[kLanes] = {};
    hipEvent_t lane_fork = nullptr;
    hipStream_t last_stream = nullptr;
    hipEvent_t batch_done = nullptr;   // recorded on last_stream when another stream needs the last batch
    bool batch_done_rec = false;
    const uint8_t* last_in = nullptr;  // device input of the last extraction
    int64_t last_pitch = 0;
    int last_images = 0, last_pairs = 0;
    double last_bf = 0.0;
    float last_fx = 0.f;
    bool have_single = false;          // orbfe_extract ran and its buffers are valid
    // per-frame stereo path (orbfe_frame_extract): both images staged in d_in (pitch frame_pitch), the
    // sheared pyramids in d_shear, every result copied into the pinned h_frame before one synchronisation
    DevBuf<uint8_t> d_shear;
    // want_pyramid == 2 (lazy): every frame's two sheared views stay in a device ring of kFrameRing slots
    // (frame serial s in slot s % kFrameRing) and reach the host only when fetched
    // (orbfe_frame_pyramid_fetch), while the serial is still in the ring
    DevBuf<uint8_t> d_ring;
    int64_t frame_serial = 0;                  // the last frame's serial (1, 2, ...)
    int64_t ring_serial[kFrameRing] = {};      // the serial whose views each slot holds (0: none)
    bool frame_ring = false;                   // the last frame put its views in the ring
    DevBuf<float> d_uin, d_uout;  // orbfe_undistort_points scratch
    HostBuf<uint8_t> h_frame;
    HostBuf<uint8_t> h_in;  // pinned staging of host images (a pageable 2-D copy goes row by row)
    int64_t frame_pitch = 0;
    bool have_frame = false, frame_pyr = false;
    size_t fo_count = 0, fo_kps = 0, fo_desc = 0, fo_uR = 0, fo_depth = 0, fo_status = 0, fo_match = 0, fo_ovf = 0,
           fo_shear = 0;

    // An executable graph may still be queued or running on the caller's stream when it is evicted or
    // dropped (nothing synchronises between batch enqueues): wait for its last launch before destroying it
    // (destroying a running executable is not specified to be safe).
    static void retire(GraphEntry& e) {
        if (e.done) {
            (void)hipEventSynchronize(e.done);
            (void)hipEventDestroy(e.done);
        }
        (void)hipGraphExecDestroy(e.exec);
    }
    void drop_graphs() {
        for (GraphEntry& e : graphs) retire(e);
        graphs.clear();
        ++gen;
    }
    ~orbfe_ctx() {
        for (GraphEntry& e : graphs) retire(e);
        if (cap_stream) (void)hipStreamDestroy(cap_stream);
        for (hipEvent_t e : prof_ev) (void)hipEventDestroy(e);
        if (own_stream) (void)hipStreamDestroy(own_stream);
        for (int k = 0; k < kLanes; ++k) {
            if (lane_stream[k]) (void)hipStreamDestroy(lane_stream[k]);
            if (lane_done[k]) (void)hipEventDestroy(lane_done[k]);
        }
        if (lane_fork) (void)hipEventDestroy(lane_fork);
        if (batch_done) (void)hipEventDestroy(batch_done);
    }
};

namespace {

// ORBextractor::ORBextractor (ORBextractor.cpp:410-470)
void build_tables(orbfe_ctx& c) {
    const orbfe_params& p = c.prm;
    if (p.nlevels < 1 || p.nlevels > kMaxLevels) throw Error(ORBFE_EINVAL, "nlevels must be in [1, 16]");
    if (p.nfeatures < 0 || !(p.scale_factor > 0.f)) throw Error(ORBFE_EINVAL, "bad nfeatures / scaleFactor");
    if (p.resize_simd_lanes != 0 && p.resize_simd_lanes != 16 && p.resize_simd_lanes != 32)
        throw Error(ORBFE_EINVAL, "resize_simd_lanes must be 0, 16 or 32");
    const int L = p.nlevels;
    c.scale_factor_d = (double)p.scale_factor;
    c.sf.assign(L, 1.0f);
    c.s2.assign(L, 1.0f);
    for (int i = 1; i < L; ++i) {
        c.sf[i] = (float)((double)c.sf[i - 1] * c.scale_factor_d);
        c.s2[i] = c.sf[i] * c.sf[i];
    }
    c.isf.resize(L);
    c.is2.resize(L);
    for (int i = 0; i < L; ++i) {
        c.isf[i] = 1.0f / c.sf[i];
        c.is2[i] = 1.0f / c.s2[i];
    }
    c.n_per_level.assign(L, 0);
    const float factor = (float)(1.0 / c.scale_factor_d);
    float want = p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; ++l) {
        c.n_per_level[l] = round_even_f(want);
        sum += c.n_per_level[l];
        want *= factor;
    }
    c.n_per_level[L - 1] = std::max(p.nfeatures - sum, 0);
    const int vmax = floor_f(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = ceil_f(kHalfPatch * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) c.umax[v] = (int)std::lrint(std::sqrt((double)kHalfPatch * kHalfPatch - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (c.umax[v0] == c.umax[v0 + 1]) ++v0;
        c.umax[v] = v0;
        ++v0;
    }
}

// Resize coefficient tables of cv::resize(INTER_LINEAR) for sw x sh -> dw x dh (8U fixed point).
void resize_tables(int sw, int sh, int dw, int dh, int simd, LevelGeo& Lg, std::vector<ResizeX>& xt,
                   std::vector<ResizeY>& yt) {
    const double inv_x = (double)dw / sw, inv_y = (double)dh / sh;
    const double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
    const int isx = (int)std::lrint(scale_x), isy = (int)std::lrint(scale_y);
    const bool area_fast = std::fabs(scale_x - isx) < DBL_EPSILON && std::fabs(scale_y - isy) < DBL_EPSILON;
    while (xt.size() % 4) xt.push_back(ResizeX{0, 0, 0});  // k_resize reads 4 entries as 2 x 16 bytes
    Lg.xtab_off = (int)xt.size();
    Lg.ytab_off = (int)yt.size();
    Lg.area = 0;
    Lg.wide = 0;
    if (area_fast && isx == 2 && isy == 2) {
        // cv::resize turns INTER_LINEAR with an exact 2x step into INTER_AREA, whose fast path
        // (resizeAreaFast_, ResizeAreaFastVec_SIMD_8u) averages 2 x 2 blocks: (a + b + c + d + 2) >> 2 over the
        // vector span (v_rshr_pack_store<2>, u16 lanes = simd / 2 per step), saturate_cast<uchar>(sum * 0.25f)
        // after it.  As linear tables: sx = 2 dx, sy = 2 dy, 2 dy + 1, all weights 1024 — the kernels' vector
        // formula (mulhi(H >> 4, b) ...) then is exactly the rounding shift, and resize_tail the half-even tail.
        Lg.area = 1;
        for (int dx = 0; dx < dw; ++dx) xt.push_back(ResizeX{2 * dx, 1024, 1024});
        Lg.xmax = dw;
        for (int k = 0; k < 4; ++k) xt.push_back(ResizeX{sw - 1, 2048, 0});  // over-read guard, as below
        const int lanes = simd / 2;
        Lg.xvec = lanes > 0 ? dw / lanes * lanes : 0;
        for (int dy = 0; dy < dh; ++dy) yt.push_back(ResizeY{2 * dy, 2 * dy + 1, 1024, 1024});
        return;
    }
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = floor_f(fx);
        fx -= sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
        }
        ResizeX r;
        r.sx = sx;
        r.a0 = sat_short(round_even_f((1.f - fx) * 2048));
        r.a1 = sat_short(round_even_f(fx * 2048));
        xt.push_back(r);
    }
    Lg.xmax = xmax;
    // over-read guard of the last group: the last column at weight 2048 (kept inside its group's byte window)
    for (int k = 0; k < 4; ++k) xt.push_back(ResizeX{sw - 1, 2048, 0});
    // k_resize gathers a 4-pixel group's taps from 8 bytes starting at the group's first sx; with steps near 2
    // (e.g. 1241 -> 620 at scaleFactor 2) the 4th pixel can fall past them: such a level is `wide` and takes
    // that pixel's taps from a window of its own (resize_tap3)
    for (int g0 = Lg.xtab_off; g0 < (int)xt.size() - 4; g0 += 4) {
        for (int k = 1; k < 4; ++k)
            if (xt[g0 + k].sx - xt[g0].sx < 0 || xt[g0 + k].sx - xt[g0].sx > (k == 3 ? 15 : 6))
                throw Error(ORBFE_EINVAL, "resize step too large for k_resize's tap windows (scale factor > ~2.3)");
        if (xt[g0 + 3].sx - xt[g0].sx > 6) Lg.wide = 1;
    }
    int xv = 0;
    if (simd > 0) {
        while (xv <= dw - simd) xv += simd;
        while (xv < dw - simd / 2) xv += simd / 2;
    }
    Lg.xvec = xv;
    auto clip = [](int v, int n) { return v >= 0 ? (v < n ? v : n - 1) : 0; };
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = floor_f(fy);
        fy -= sy;
        ResizeY r;
        r.sy0 = clip(sy, sh);
        r.sy1 = clip(sy + 1, sh);
        r.b0 = sat_short(round_even_f((1.f - fy) * 2048));
        r.b1 = sat_short(round_even_f(fy * 2048));
        yt.push_back(r);
    }
}

// k_octree (bins) tables of level L (DistributeOctTree, ORBextractor.cpp:539-762).  ExtractorNode::DivideNode
// splits a box at mx = x0 + ceil((x1 - x0) / 2), my likewise, and a key goes right / down iff x >= mx /
// y >= my (:483-509): the x splits a key meets depend only on its column's x interval and its own x, the y
// splits only on [0, span_y] and its y.  So a key's quadrant at every depth is a table lookup:
// X[x_rel] = column << 2D | x bits at the even positions, Y[y_rel] = y bits at the odd positions, and
// code = X | Y is the key's whole path in Morton order (digit q = x bit + 2 y bit at bits 2 (D - depth)).
// D is the least depth at which every two distinct pixels of a column differ in their path, so a node of
// depth D holds one key and is never divided.  The initial column is (int)((float)x / hX), clamped to
// nIni - 1, and column i's box is [(int)(hX * i), (int)(hX * (i + 1))] x [0, span_y] (:543-584).
void octree_tables(LevelGeo& L, int n_feat, std::vector<uint32_t>& tab) {
    L.oct_d = L.oct_d0 = L.oct_bins = 0;
    L.oct_nx = L.span_x + 1;
    L.oct_ny = L.span_y + 1;
    if (L.ncell == 0 || L.n_ini <= 0) {
        L.oct_xt = L.oct_yt = (int)tab.size();
        return;
    }
    constexpr int kDmax = 15;
    auto xpath = [&](int x, int* col) {  // kDmax x bits, MSB = depth 1
        int ci = std::min((int)((float)x / L.hx), L.n_ini - 1);
        *col = ci;
        int x0 = (int)(L.hx * (float)ci), x1 = (int)(L.hx * (float)(ci + 1));
        uint32_t b = 0;
        for (int d = 0; d < kDmax; ++d) {
            const int mx = x0 + ((x1 - x0 + 1) >> 1);
            const bool r = x >= mx;
            b = (b << 1) | (uint32_t)r;
            if (r) x0 = mx; else x1 = mx;
        }
        return b;
    };
    auto ypath = [&](int y) {
        int y0 = 0, y1 = L.span_y;
        uint32_t b = 0;
        for (int d = 0; d < kDmax; ++d) {
            const int my = y0 + ((y1 - y0 + 1) >> 1);
            const bool r = y >= my;
            b = (b << 1) | (uint32_t)r;
            if (r) y0 = my; else y1 = my;
        }
        return b;
    };
    std::vector<uint32_t> xp(L.oct_nx), yp(L.oct_ny);
    std::vector<int> xc(L.oct_nx);
    for (int x = 0; x < L.oct_nx; ++x) xp[x] = xpath(x, &xc[x]);
    for (int y = 0; y < L.oct_ny; ++y) yp[y] = ypath(y);
    // least D separating neighbours (paths are monotone in x / y, so neighbours suffice).  Only coordinates
    // a key can take matter: a FAST cell's keys lie in its ROI minus the 3-px circle border, so x_rel <=
    // span_x - 4 and y_rel <= span_y - 4 (ORBextractor.cpp:788-824); the table's last entries (which the
    // float column split can leave outside their column's box, e.g. 2460 px wide, level 5) only clamp.
    int D = 1;
    const int kx = std::max(1, L.oct_nx - 4), ky = std::max(1, L.oct_ny - 4);
    for (int x = 1; x < kx; ++x)
        if (xc[x] == xc[x - 1]) {
            const uint32_t d = xp[x] ^ xp[x - 1];
            if (!d) throw Error(ORBFE_EINVAL, "octree tables: two columns of a level share a path");
            D = std::max(D, kDmax - (31 - __builtin_clz(d)));
        }
    for (int y = 1; y < ky; ++y) {
        const uint32_t d = yp[y] ^ yp[y - 1];
        if (!d) throw Error(ORBFE_EINVAL, "octree tables: two rows share a path");
        D = std::max(D, kDmax - (31 - __builtin_clz(d)));
    }
    int cb = 0;
    while ((1 << cb) < L.n_ini) ++cb;
    if (D >= kDmax || 2 * D + cb > 32) throw Error(ORBFE_EINVAL, "octree tables: level too large for 32-bit paths");
    // bins: depth D0 with about 8 N nodes' worth of bins, at most 2048 (the nodes the octree ends with sit
    // at depth <= 4 on every KITTI / EuRoC / synthetic image measured; deeper divisions take the
    // per-candidate path of the kernel)
    int D0 = 1;
    while (D0 < D && (int64_t)L.n_ini << (2 * D0) < 8 * (int64_t)std::max(n_feat, 1)) ++D0;
    while (D0 > 1 && ((int64_t)L.n_ini << (2 * D0)) > 2048) --D0;
    L.oct_d = D;
    L.oct_d0 = D0;
    L.oct_bins = L.n_ini << (2 * D0);
    L.oct_xt = (int)tab.size();
    for (int x = 0; x < L.oct_nx; ++x) {
        uint32_t s = 0;
        for (int d = 1; d <= D; ++d)
            if ((xp[x] >> (kDmax - d)) & 1u) s |= 1u << (2 * (D - d));
        tab.push_back(((uint32_t)xc[x] << (2 * D)) | s);
    }
    L.oct_yt = (int)tab.size();
    for (int y = 0; y < L.oct_ny; ++y) {
        uint32_t s = 0;
        for (int d = 1; d <= D; ++d)
            if ((yp[y] >> (kDmax - d)) & 1u) s |= 1u << (2 * (D - d) + 1);
        tab.push_back(s);
    }
}

// The divisor of a level's packed keys (kKeyXYBits, key_xy in the kernels): y = mul_hi(xy, kmag) >> ksh ==
// floor(xy / w) for every xy < 2^24 with kmag = ceil(2^(31 + s) / w), ksh = s - 1, s = ceil(log2 w) (kmag < 2^32
// because w > 2^(s - 1); exact because the error term xy * (kmag * w - 2^(31 + s)) < 2^24 * w < 2^(31 + s)).
// Checked here on the level's extreme and row-boundary indices.  A 1-px-wide level has no FAST cells, hence no
// keys: its divisor only has to exist.
void key_divisor(LevelGeo& L) {
    const uint32_t w = (uint32_t)L.w;
    if (w < 2) {
        L.kmag = 0;
        L.ksh = 0;
        return;
    }
    int s = 0;
    while ((1u << s) < w) ++s;
    const unsigned __int128 num = (unsigned __int128)1 << (31 + s);
    const uint64_t mag = (uint64_t)((num + w - 1) / w);
    if (mag > 0xFFFFFFFFull) throw Error(ORBFE_EINVAL, "key divisor out of range");
    L.kmag = (uint32_t)mag;
    L.ksh = s - 1;
    const uint32_t n = w * (uint32_t)L.h;
    for (uint32_t y : {0u, 1u, (uint32_t)L.h / 2, (uint32_t)L.h - 1})
        for (int64_t d : {(int64_t)-1, (int64_t)0, (int64_t)1, (int64_t)w - 1}) {
            const int64_t v = (int64_t)y * w + d;
            if (v < 0 || v >= (int64_t)n) continue;
            const uint32_t q = (uint32_t)(((uint64_t)(uint32_t)v * L.kmag) >> 32) >> L.ksh;
            if (q != (uint32_t)v / w) throw Error(ORBFE_EINVAL, "key divisor check failed");
        }
}

void build_geometry(orbfe_ctx& c, int W, int H) {
    const int L = c.prm.nlevels;
    Geo& g = c.geo;
    std::memset(&g, 0, sizeof(g));
    g.nlevels = L;
    g.W = W;
    g.H = H;
    g.ini_th = std::min(std::max(c.prm.ini_th_fast, 0), 255);  // cv::FAST clamps the threshold
    g.min_th = std::min(std::max(c.prm.min_th_fast, 0), 255);
    for (int v = 0; v < 16; ++v) g.umax[v] = c.umax[v];
    c.cells.clear();
    c.xt.clear();
    c.yt.clear();
    c.octab.clear();
    c.maxcell = 0;
    int64_t ws = 0, shear = 0;
    int kp_off = 0, key_off = 0;
    int64_t slot_off = 0;
    for (int l = 0; l < L; ++l) {
        LevelGeo& Lg = g.lv[l];
        g.scale[l] = c.sf[l];
        g.inv_scale[l] = c.isf[l];
        Lg.scale = c.sf[l];
        Lg.inv_scale = c.isf[l];
        Lg.w = round_even_f((float)W * c.isf[l]);
        Lg.h = round_even_f((float)H * c.isf[l]);
        // the packed level keys (FAST slots, key cache, level keypoints: (x + y * w) | score << 24) hold a
        // pixel's row-major index in 24 bits (kKeyXYBits): every level of at most 2^24 pixels
        if (Lg.w < 1 || Lg.h < 1) throw Error(ORBFE_EINVAL, "level size out of range (empty level)");
        if ((int64_t)Lg.w * Lg.h > (int64_t)1 << kKeyXYBits || Lg.w > kMaxCellCoord || Lg.h > kMaxCellCoord)
            throw Error(ORBFE_EINVAL, "level " + std::to_string(l) + " (" + std::to_string(Lg.w) + "x" + std::to_string(Lg.h) +
                                          ") has more than 2^24 pixels (or a side above 32 767 px): its pixel index does "
                                          "not fit the 24 bits of a packed level key");
        key_divisor(Lg);
        // levels of 19 px or less are padded by an iterated reflection (k_shear); they have no FAST cells
        Lg.pitch = (Lg.w + 15) & ~15;
        if (l > 0) {
            Lg.ws_off = ws;
            ws += ((int64_t)Lg.pitch * Lg.h + 255) & ~(int64_t)255;
            resize_tables(g.lv[l - 1].w, g.lv[l - 1].h, Lg.w, Lg.h, c.prm.resize_simd_lanes, Lg, c.xt, c.yt);
        }
        Lg.shear_off = shear;
        shear += ((int64_t)Lg.w * Lg.h + 3) & ~(int64_t)3;
        Lg.n_feat = c.n_per_level[l];
        Lg.size = (float)(int)(31 * c.sf[l]);
        // cell grid (ORBextractor.cpp:772-806)
        const int minX = kBorder, minY = kBorder, maxX = Lg.w - kEdge + 3, maxY = Lg.h - kEdge + 3;
        Lg.span_x = maxX - minX;
        Lg.span_y = maxY - minY;
        const float width = (float)(maxX - minX), height = (float)(maxY - minY);
        const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
        Lg.cell0 = (int)c.cells.size();
        Lg.key_off = key_off;
        int key_cap = 0;
        if (nCols > 0 && nRows > 0) {
            const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
            for (int i = 0; i < nRows; ++i) {
                const float iniY = (float)(minY + i * hCell);
                float maxYc = iniY + hCell + 6;
                if (iniY >= maxY - 3) continue;
                if (maxYc > maxY) maxYc = (float)maxY;
                for (int j = 0; j < nCols; ++j) {
                    const float iniX = (float)(minX + j * wCell);
                    float maxXc = iniX + wCell + 6;
                    if (iniX >= maxX - 6) continue;
                    if (maxXc > maxX) maxXc = (float)maxX;
                    CellGeo cg{};
                    cg.level = (int16_t)l;
                    cg.kw = (int16_t)Lg.w;
                    cg.x0 = (int16_t)(int)iniX;
                    cg.y0 = (int16_t)(int)iniY;
                    cg.x1 = (int16_t)(int)maxXc;
                    cg.y1 = (int16_t)(int)maxYc;
                    const int rw = cg.x1 - cg.x0, rh = cg.y1 - cg.y0;
                    // k_detect stages a ROI row from column -1 as <= 16 dwords, one per lane of a 16-lane DPP row
                    if (rw > 59 || rh > 64) throw Error(ORBFE_EINVAL, "FAST cell ROI larger than 59 x 64 px");
                    if (cg.x0 < 1) throw Error(ORBFE_EINVAL, "FAST cell ROI at column 0");
                    const int ww = std::max(rw - 6, 0), wh = std::max(rh - 6, 0);
                    g.max_rh = std::max(g.max_rh, rh);
                    g.max_rw = std::max(g.max_rw, rw);
                    g.max_wh = std::max(g.max_wh, wh);
                    g.max_win = std::max(g.max_win, (ww * wh + 15) & ~15);
                    g.fd_mp = std::max(g.fd_mp, (ww + 6 + 15) & ~15);
                    cg.slot_off = (int)slot_off;
                    cg.slot_cap = ((ww + 1) / 2) * ((wh + 1) / 2);
                    g.fd_pq = std::max(g.fd_pq, (((ww + 1) / 2) * wh + 7) & ~7);
                    g.fd_alt = std::max(g.fd_alt, cg.slot_cap);
                    slot_off += cg.slot_cap;
                    key_cap += cg.slot_cap;
                    c.cells.push_back(cg);
                }
            }
        }
        Lg.ncell = (int)c.cells.size() - Lg.cell0;
        Lg.key_cap = key_cap;
        key_off += (key_cap + 3) & ~3;  // 16-byte aligned levels (k_octree_bins reads its key cache as dwordx4)
        c.maxcell = std::max(c.maxcell, Lg.ncell);
        if (key_cap >= (1 << 24)) throw Error(ORBFE_EINVAL, "too many FAST candidates per level");
        // DistributeOctTree initial columns (:543-545)
        Lg.n_ini = 0;
        Lg.hx = 1.f;
        {
            // the reference runs DistributeOctTree on every level, cells or not: nIni = round((float)spanX /
            // spanY) sizes vpIniNodes.resize(nIni) (:543-550), which throws std::length_error for nIni < 0 (a
            // level lower than 32 px but wider, e.g. 1241x376 at scaleFactor 2 from its 5th level on) and is
            // undefined for spanY == 0 (float division by zero): such geometries are refused like the
            // reference refuses them.  Smaller levels pass (e.g. square ones: nIni = 1).
            const float q = Lg.span_y != 0 ? std::round((float)Lg.span_x / (float)Lg.span_y) : NAN;
            if (!std::isfinite(q) || q < 0.f)
                throw Error(ORBFE_EINVAL, "level " + std::to_string(l) + " (" + std::to_string(Lg.w) + "x" +
                                              std::to_string(Lg.h) + "): the reference's DistributeOctTree fails "
                                              "(vpIniNodes.resize(nIni) with nIni = round(spanX / spanY) negative or "
                                              "undefined, ORBextractor.cpp:543-550)");
        }
        if (Lg.ncell > 0) {
            if (Lg.span_y <= 0 || Lg.span_x <= 0) throw Error(ORBFE_EINVAL, "degenerate level");
            Lg.n_ini = (int)std::round((float)Lg.span_x / Lg.span_y);
            if (Lg.n_ini <= 0)
                throw Error(ORBFE_EINVAL, "level " + std::to_string(l) + " (" + std::to_string(Lg.w) + "x" +
                                              std::to_string(Lg.h) + "): the reference's DistributeOctTree indexes "
                                              "vpIniNodes out of range (nIni = round(spanX / spanY) = 0 with FAST cells, "
                                              "ORBextractor.cpp:543-568)");
            Lg.hx = (float)Lg.span_x / Lg.n_ini;
        }
        Lg.kp_cap = std::max(Lg.n_feat + 2, 4 * Lg.n_ini) + 2;
        octree_tables(Lg, Lg.n_feat, c.octab);
        g.oct_bins_max = std::max(g.oct_bins_max, Lg.oct_bins);
        g.oct_tab_max = std::max(g.oct_tab_max, Lg.oct_nx + Lg.oct_ny);
        g.oct_kblk_max = std::max(g.oct_kblk_max, std::min((Lg.key_cap >> kObKblkSh) + 1, kObKblkMax));
        Lg.kp_off = kp_off;
        kp_off += Lg.kp_cap;
        g.max_ncap = std::max(g.max_ncap, Lg.kp_cap);
    }
    g.ncells = (int)c.cells.size();
    g.kp_cap = kp_off;
    g.lvl_kp_cap = kp_off;
    // k_resize geometry: source rows per kRsRows-row output band, source row stride, groups per row
    g.rs_nsrc = 1;
    g.rs_sp = g.W;
    g.rs_ngrp = 4;
    for (int l = 1; l < L; ++l) {
        LevelGeo& Lg = g.lv[l];
        Lg.rs_sp = l >= 2 ? g.lv[l - 1].pitch : g.W;
        // the band's source rows are staged whole (k_resize_rows' dynamic LDS: nsrc x sp bytes): a level so wide
        // that 16-row bands would not fit takes 8-, 4-, 2- or 1-row bands (round 6; 16 up to ~7 000 px)
        for (Lg.rs_rows = kRsRows;; Lg.rs_rows /= 2) {
            Lg.rs_nsrc = 1;
            for (int dy0 = 0; dy0 < Lg.h; dy0 += Lg.rs_rows) {
                const int dy1 = std::min(dy0 + Lg.rs_rows, Lg.h);
                Lg.rs_nsrc = std::max(Lg.rs_nsrc, c.yt[Lg.ytab_off + dy1 - 1].sy1 - c.yt[Lg.ytab_off + dy0].sy0 + 1);
            }
            if ((int64_t)Lg.rs_nsrc * Lg.rs_sp + 16 <= 150 * 1024 || Lg.rs_rows == 1) break;
        }
        if ((int64_t)Lg.rs_nsrc * Lg.rs_sp + 16 > 150 * 1024)
            throw Error(ORBFE_EINVAL, "image too wide for the k_resize band staging (LDS)");
        Lg.rs_ngrp = ((Lg.w + 3) / 4 + 3) & ~3;
        g.rs_nsrc = std::max(g.rs_nsrc, Lg.rs_nsrc);
        g.rs_sp = std::max(g.rs_sp, Lg.rs_sp);
        g.rs_ngrp = std::max(g.rs_ngrp, Lg.rs_ngrp);
    }
    g.ws_bytes = std::max<int64_t>(ws, 256);
    g.shear_bytes = shear;
    g.slot_total = std::max<int64_t>(slot_off, 1);
    g.key_total = std::max(key_off, 4);
    if (g.max_ncap >= 65535) throw Error(ORBFE_EINVAL, "nfeatures too large for the octree node index");
    // octree kernel: k_octree_bins unless its LDS carve exceeds 150 KiB (or the caller forces the
    // per-candidate k_octree, orbfe_set_octree_kernel); k_octree keeps the candidates in LDS when the node
    // arrays leave room for them, else in the global scratch (very large per-level feature counts)
    g.oct_v = c.octree_force ? 1 : 0;
    if (g.oct_v == 0 && octree_bins_lds_bytes(g, c.maxcell) > 150 * 1024) g.oct_v = 1;
    g.oct_keys = kOctKeys;
    if (octree_lds_bytes(g, c.maxcell) > 150 * 1024) g.oct_keys = 0;
    if (octree_lds_bytes(g, c.maxcell) > 150 * 1024)
        throw Error(ORBFE_EINVAL, "octree LDS footprint exceeds the 160 KiB LDS of a CU (nfeatures per level too large)");
    c.W = W;
    c.H = H;
}

// k_orb's per-lane tables (see k_orb in orbfe_kernels.hip).  Horizontal items: the (row pair m, 4-column
// group gx) of the 43 x 40 horizontally blurred window that some BRIEF sample's 7 vertical taps read; a
// sample lies at (row, col) with row^2 + col^2 <= (18.385 + 0.708)^2 (the pattern's largest radius,
// ORBextractor.cpp:150-408, plus rint's rounding), blurred row o = row + 18 reads H rows o .. o + 6 at column
// col + 21.  Centroid slots: every dword of staged rows 6 .. 36 that holds a byte of the umax disc
// (ORBextractor.cpp:77-104), with the signed byte weights u (m10) and v (m01) of its disc bytes (0 elsewhere).
std::vector<uint32_t> orb_tables(const int* umax) {
    std::vector<uint32_t> t(kOrbTabWords, 0u);
    bool need[44][40] = {};
    const double R = 18.384776310850235 + 0.7072;
    for (int row = -18; row <= 18; ++row)
        for (int col = -18; col <= 18; ++col)
            if (row * row + col * col <= R * R)
                for (int k = 0; k < 7; ++k) need[row + 18 + k][col + 21] = true;
    int n = 0;
    for (int m = 0; m < 22; ++m)
        for (int gx = 0; gx < 10; ++gx) {
            bool any = false;
            for (int rr = 0; rr < 2; ++rr)
                for (int c = 0; c < 4; ++c) any |= need[2 * m + rr][4 * gx + c];
            if (!any) continue;
            if (n >= 192) throw Error(ORBFE_EINVAL, "k_orb: more than 192 horizontal items");
            t[n++] = (uint32_t)(2 * m * 12 + gx) | ((uint32_t)(m * 10 + gx) << 16);
        }
    // lanes without an item run a dummy one: source dword 0, H slot (row pair 0, group 0) — a corner of the
    // window no BRIEF sample reaches, so k_orb needs no per-item test
    for (int rr = 0; rr < 2; ++rr)
        for (int c = 0; c < 4; ++c)
            if (need[rr][c]) throw Error(ORBFE_EINVAL, "k_orb: the dummy H slot lies on the sample disc");
    for (; n < 192; ++n) t[n] = 0u;
    uint32_t* cw = t.data() + 192;
    int sl = 0;
    for (int r = 0; r < 31; ++r) {
        const int v = r - kHalfPatch, um = umax[v < 0 ? -v : v];
        for (int d = (17 - um) / 4; d <= (um + 17) / 4; ++d) {
            if (sl >= 256) throw Error(ORBFE_EINVAL, "k_orb: more than 256 centroid slots");
            uint32_t wu = 0, wv = 0;  // signed byte weights u and v of the disc's bytes, 0 off the disc
            for (int b = 0; b < 4; ++b) {
                const int u = 4 * d + b - 17;
                if (u >= -um && u <= um) {
                    wu |= (uint32_t)(uint8_t)(int8_t)u << (8 * b);
                    wv |= (uint32_t)(uint8_t)(int8_t)v << (8 * b);
                }
            }
            cw[4 * sl] = wu;
            cw[4 * sl + 1] = wv;
            cw[4 * sl + 2] = (uint32_t)((6 + r) * 12 + 2 + d);
            cw[4 * sl + 3] = 0u;
            ++sl;
        }
    }
    return t;
}

// Every call that enqueues work on (or reallocates) the handle's device buffers ends the validity of the
// results an earlier orbfe_extract / orbfe_frame_extract left there: the getters of those results then
// fail with ORBFE_ESTATE instead of reading buffers, offsets and a geometry that no longer belong together.
void invalidate_results(orbfe_ctx& c) {
    c.have_single = false;
    c.have_frame = false;
    c.frame_pyr = false;
}

// Per-kernel attributes (dynamic LDS above 64 KiB) are set here, when the geometry is built, and never
// inside an enqueue: a graph capture (orbfe_set_graphs) records only stream work.
void prepare_kernels(orbfe_ctx& c) { HIPCK(prepare_octree(c.geo, c.maxcell)); }

void reserve(orbfe_ctx& c, int W, int H, int max_images) {
    if (W <= 0 || H <= 0 || max_images <= 0) throw Error(ORBFE_EINVAL, "bad reserve geometry");
    if (W != c.W || H != c.H) {
        invalidate_results(c);
        c.drop_graphs();
        c.cascades.clear();
        for (int64_t& r : c.ring_serial) r = 0;  // no earlier frame's views survive a geometry change
        build_geometry(c, W, H);
        c.max_images = 0;
        c.d_cells.ensure(c.cells.size());
        HIPCK(hipMemcpy(c.d_cells.p, c.cells.data(), c.cells.size() * sizeof(CellGeo), hipMemcpyHostToDevice));
        {
            const std::vector<uint32_t> ot = orb_tables(c.umax);
            c.d_orb.ensure(ot.size());
            HIPCK(hipMemcpy(c.d_orb.p, ot.data(), ot.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
        c.d_xt.ensure(c.xt.size());
        if (!c.xt.empty())
            HIPCK(hipMemcpy(c.d_xt.p, c.xt.data(), c.xt.size() * sizeof(ResizeX), hipMemcpyHostToDevice));
        c.d_yt.ensure(c.yt.size());
        if (!c.yt.empty())
            HIPCK(hipMemcpy(c.d_yt.p, c.yt.data(), c.yt.size() * sizeof(ResizeY), hipMemcpyHostToDevice));
        c.d_octab.ensure(std::max<size_t>(c.octab.size(), 1));
        if (!c.octab.empty())
            HIPCK(hipMemcpy(c.d_octab.p, c.octab.data(), c.octab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        prepare_kernels(c);
    }
    if (max_images > c.max_images) {
        invalidate_results(c);  // the per-image buffers may move
        c.drop_graphs();
        const Geo& g = c.geo;
        const size_t n = (size_t)max_images;
        c.d_ws.ensure(n * g.ws_bytes);
        c.d_cell_count.ensure(n * std::max(g.ncells, 1));
        c.d_slots.ensure(n * g.slot_total);
        c.d_kd.ensure(n * g.key_total);
        c.d_kn.ensure(n * g.key_total);
        c.d_lvl_kp.ensure(n * g.lvl_kp_cap);
        c.d_lvl_count.ensure(n * g.nlevels);
        c.d_kps.ensure(n * g.kp_cap);
        c.d_desc.ensure(n * g.kp_cap * 32);
        c.d_count.ensure(n);
        c.d_overflow.ensure(1);
        const size_t np = n / 2 + 1;
        c.d_uR.ensure(np * g.kp_cap);
        c.d_depth.ensure(np * g.kp_cap);
        c.d_status.ensure(np * g.kp_cap);
        c.d_match.ensure(np * g.kp_cap);
        // a right keypoint covers at most ceil(y+2s) - floor(y-2s) + 1 <= 4 s_max + 3 rows
        c.bucket_cap = (int64_t)g.kp_cap * (int64_t)(4 * c.sf[g.nlevels - 1] + 4);
        c.d_boff.ensure(np * (g.H + 1));
        c.d_bidx.ensure(np * c.bucket_cap);
        c.d_rinfo.ensure(np * g.kp_cap);
        c.max_images = max_images;
    }
}

// record event `k` of the current profiled batch on the launch stream: 0 start, 1 after resize, 2 after
// detect, 3 after octree, 4 after describe (k_orb), 5 after stereo.
void prof_mark(orbfe_ctx& c, hipStream_t s, int k) {
    if (!c.prof_on || c.prof_n >= c.prof_max) return;
    HIPCK(hipEventRecord(c.prof_ev[(size_t)c.prof_n * kProfEvents + k], s));
}

// Images [i0, i0 + n) of the batch: every per-image buffer is passed at the chunk's offset, the
// kernels index images from there.  prof: record stage boundaries on s.
// k_resize_cascade strips (see the kernel): S strips of the top level's rows, and below it, level by level,
// the rows strip s owns (a partition: the first source row of its next-level rows onwards) and the rows it
// computes (its own plus the source rows of the next level's computed rows).  Null when the LDS the strips
// need exceeds 150 KiB.
std::unique_ptr<orbfe_ctx::Cascade> resize_strips(const orbfe_ctx& c, int S) {
    const Geo& g = c.geo;
    const int L = g.nlevels, top = L - 1;
    if (L < 2 || S < 1 || S > g.lv[top].h) return nullptr;
    std::vector<std::vector<int>> own(L, std::vector<int>(S + 1)), clo(L, std::vector<int>(S)), chi(L, std::vector<int>(S));
    for (int k = 0; k <= S; ++k) own[top][k] = (int)((int64_t)k * g.lv[top].h / S);
    auto yt = [&](int l, int dy) -> const ResizeY& { return c.yt[g.lv[l].ytab_off + dy]; };
    for (int l = top - 1; l >= 1; --l) {
        own[l][0] = 0;
        own[l][S] = g.lv[l].h;
        for (int k = 1; k < S; ++k) own[l][k] = yt(l + 1, own[l + 1][k]).sy0;
    }
    for (int k = 0; k < S; ++k) {
        clo[top][k] = own[top][k];
        chi[top][k] = own[top][k + 1];
        if (chi[top][k] <= clo[top][k]) return nullptr;
        for (int l = top - 1; l >= 1; --l) {
            clo[l][k] = std::min(own[l][k], yt(l + 1, clo[l + 1][k]).sy0);
            chi[l][k] = std::max(own[l][k + 1], yt(l + 1, chi[l + 1][k] - 1).sy1 + 1);
        }
    }
    size_t A = 0, B = 0;
    std::vector<int16_t> tab((size_t)S * L * 4, 0);
    for (int k = 0; k < S; ++k) {
        const int ys_lo = yt(1, clo[1][k]).sy0, ys_hi = yt(1, chi[1][k] - 1).sy1;
        A = std::max(A, (size_t)(ys_hi - ys_lo + 1) * g.W + 8);  // the staged level-0 run (+ misalignment)
        for (int l = 1; l < L; ++l) {
            const size_t b = (size_t)(chi[l][k] - clo[l][k]) * g.lv[l].pitch;
            (l & 1 ? B : A) = std::max(l & 1 ? B : A, b);
            int16_t* e = &tab[((size_t)k * L + l) * 4];
            e[0] = (int16_t)clo[l][k];
            e[1] = (int16_t)chi[l][k];
            e[2] = (int16_t)own[l][k];
            e[3] = (int16_t)own[l][k + 1];
        }
    }
    auto a16 = [](size_t v) { return (v + 16 + 15) & ~(size_t)15; };  // + the taps' 12-byte over-read
    std::unique_ptr<orbfe_ctx::Cascade> cs(new orbfe_ctx::Cascade());
    cs->S = S;
    cs->off_b = (int)a16(A);
    cs->off_x = cs->off_b + (int)a16(B);
    cs->lds = cs->off_x + (int)((size_t)g.rs_ngrp * 72);  // two levels' x entries (k_resize_cascade prefetch)
    if (cs->lds > 150 * 1024) return nullptr;
    cs->tab.ensure(tab.size());
    HIPCK(hipMemcpy(cs->tab.p, tab.data(), tab.size() * sizeof(int16_t), hipMemcpyHostToDevice));
    HIPCK(prepare_resize_cascade(cs->lds));
    return cs;
}

// Pyramid of an n-image enqueue: the one-launch cascade for small batches (< kCascadeImages images; strips
// for >= ~512 workgroups, at least 3 top-level rows each), else the per-level k_resize_rows launches.  Built
// (uploads, kernel attributes) before an enqueue is captured: prepare_pyramid runs outside the capture.
constexpr int kCascadeImages = kSmallBatchImages;

// compute units of the current device (one strip workgroup per CU: a 1 024-thread strip is a latency chain,
// and two of them on one CU run at half speed each)
// (atomic entries: handles on several threads may ask at once; a race only repeats the same query)
static int device_cus() {
    static std::atomic<int> cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int v = cus[dev].load(std::memory_order_relaxed);
    if (!v) {
        int a = 0;
        v = hipDeviceGetAttribute(&a, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && a > 0 ? a : 256;
        cus[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

// strips per image: at most one workgroup per CU for the batch (8 images on 256 CUs: 32 strips, not 35 of which
// 24 CUs would hold two: 33 -> ~20 us), at least 3 top-level rows each, at least 4 strips
int cascade_strips(const orbfe_ctx& c, int n) {
    if (c.cascade_force) return c.cascade_force;
    if (n >= kCascadeImages || c.geo.nlevels < 2) return -1;
    const int htop = c.geo.lv[c.geo.nlevels - 1].h;
    return std::max(4, std::min(device_cus() / std::max(n, 1), std::max(4, htop / 3)));
}

orbfe_ctx::Cascade* find_cascade(orbfe_ctx& c, int S) {
    for (auto& cs : c.cascades)
        if (cs->S == S) return cs.get();
    return nullptr;
}

void prepare_pyramid(orbfe_ctx& c, int n) {
    for (int S = cascade_strips(c, n); S > 0 && !find_cascade(c, S); S += 4) {  // more strips need less LDS
        std::unique_ptr<orbfe_ctx::Cascade> cs = resize_strips(c, S);
        if (cs) {
            c.cascades.push_back(std::move(cs));
            return;
        }
        if (S > c.geo.lv[c.geo.nlevels - 1].h) return;
    }
}

// zero_ovf: the batch's overflow word is cleared by the first pyramid launch instead of a separate memset
// (one stream operation less in front of the chain); only for an enqueue that owns the word alone (not the
// concurrent chunks of orbfe_set_lanes, one of which could clear a bound another chunk already flagged).
// bucket: the stereo arguments of the range's pairs (n / 2 of them) when k_orb's launch is to build their row
// buckets too (the front-end enqueues; orb_fuses_bucket)
void extract_range(orbfe_ctx& c, const uint8_t* d_in, int64_t pitch, int i0, int n, hipStream_t s, bool prof,
                   int lane = -1, bool zero_ovf = false, const StereoArgs* bucket = nullptr) {
    const Geo& g = c.geo;
    const uint8_t* in = d_in + (int64_t)i0 * pitch;
    uint8_t* ws = c.d_ws.p + (int64_t)i0 * g.ws_bytes;
    int* cell_count = c.d_cell_count.p + (int64_t)i0 * g.ncells;
    uint32_t* slots = c.d_slots.p + (int64_t)i0 * g.slot_total;
    uint32_t* kd = c.d_kd.p + (int64_t)i0 * g.key_total;
    uint16_t* kn = c.d_kn.p + (int64_t)i0 * g.key_total;
    uint32_t* lvl_kp = c.d_lvl_kp.p + (int64_t)i0 * g.lvl_kp_cap;
    int* lvl_count = c.d_lvl_count.p + (int64_t)i0 * g.nlevels;
    orbfe_keypoint* kps = c.d_kps.p + (int64_t)i0 * g.kp_cap;
    uint8_t* desc = c.d_desc.p + (int64_t)i0 * g.kp_cap * 32;
    int* count = c.d_count.p + i0;
    if (prof) prof_mark(c, s, 0);
    if (zero_ovf && g.nlevels < 2) HIPCK(hipMemsetAsync(c.d_overflow.p, 0, sizeof(int), s));
    int S = cascade_strips(c, n);
    orbfe_ctx::Cascade* cs = nullptr;
    while (S > 0 && !(cs = find_cascade(c, S)) && S <= g.lv[g.nlevels - 1].h) S += 4;  // prepare_pyramid's choice
    if (cs) {
        HIPCK(launch_resize_cascade(g, in, pitch, ws, c.d_xt.p, c.d_yt.p, cs->tab.p, cs->S, cs->off_b, cs->off_x, cs->lds,
                                    n, s, zero_ovf ? c.d_overflow.p : nullptr));
    } else {
        for (int l = 1; l < g.nlevels; ++l)
            HIPCK(launch_resize(g, l, in, pitch, ws, c.d_xt.p, c.d_yt.p, n, s, 0,
                                zero_ovf && l == 1 ? c.d_overflow.p : nullptr));
    }
    if (prof) prof_mark(c, s, 1);
    (void)lane;
    if (g.ncells > 0) HIPCK(launch_detect(g, c.d_cells.p, in, pitch, ws, cell_count, slots, n, s));
    if (prof) prof_mark(c, s, 2);
    HIPCK(launch_octree(g, c.d_cells.p, cell_count, slots, c.d_octab.p, kd, kn, lvl_kp, lvl_count, c.d_overflow.p,
                        c.maxcell, n, s));
    if (prof) prof_mark(c, s, 3);
    HIPCK(launch_orb(g, in, pitch, ws, lvl_kp, lvl_count, kps, desc, count, n, c.d_orb.p, s, 0, bucket, bucket ? n / 2 : 0));
    if (prof) prof_mark(c, s, 4);
}

void check_extract(orbfe_ctx& c, int64_t pitch, int n) {
    const Geo& g = c.geo;
    if (n > c.max_images) throw Error(ORBFE_ECAPACITY, "batch larger than the reserved image count");
    if (pitch < (int64_t)g.W * g.H) throw Error(ORBFE_EINVAL, "image pitch smaller than width*height");
}

void enqueue_extract(orbfe_ctx& c, const uint8_t* d_in, int64_t pitch, int n, hipStream_t s) {
    if (n <= 0) return;
    check_extract(c, pitch, n);
    prepare_pyramid(c, n);
    extract_range(c, d_in, pitch, 0, n, s, true, -1, true);
    c.last_in = d_in;
    c.last_pitch = pitch;
    c.last_images = n;
    c.last_stream = s;
}

void stereo_buffers(orbfe_ctx& c, StereoArgs& a, int p0) {
    a.bucket_off = c.d_boff.p + (int64_t)p0 * (c.geo.H + 1);
    a.bucket_idx = c.d_bidx.p + (int64_t)p0 * c.bucket_cap;
    a.bucket_cap = c.bucket_cap;
    a.rinfo = c.d_rinfo.p + (int64_t)p0 * c.geo.kp_cap;
}

void stereo_consts(double bf, float fx, StereoArgs& a) {
    const float bf32 = (float)bf;                 // NEP 50: the Python float meets an np.float32
    const float mb = bf32 / fx;                   // Frame.py:43  mbf / mK[0][0]
    a.maxD = bf32 / mb;                           // Frame.py:183 mbf / minZ
    a.bf32 = bf32;
    a.bf = bf;
}

// Stereo arguments of pairs [p0, ...) (images 2p, 2p + 1) of the batch at d_in.
StereoArgs stereo_args(orbfe_ctx& c, const uint8_t* d_in, int64_t pitch, int p0, double bf, float fx) {
    const Geo& g = c.geo;
    const int64_t i0 = 2 * (int64_t)p0;
    StereoArgs a{};
    a.kpsL = c.d_kps.p + i0 * g.kp_cap;
    a.kpsR = a.kpsL + g.kp_cap;
    a.kp_stride = 2 * (int64_t)g.kp_cap;
    a.descL = c.d_desc.p + i0 * g.kp_cap * 32;
    a.descR = a.descL + (int64_t)g.kp_cap * 32;
    a.countL = c.d_count.p + i0;
    a.countR = a.countL + 1;
    a.cnt_stride = 2;
    a.lvl0L = d_in + i0 * pitch;
    a.lvl0R = a.lvl0L + pitch;
    a.lvl0_stride = 2 * pitch;
    a.wsL = c.d_ws.p + i0 * g.ws_bytes;
    a.wsR = a.wsL + g.ws_bytes;
    a.ws_stride = 2 * g.ws_bytes;
    a.u_right = c.d_uR.p + (int64_t)p0 * g.kp_cap;
    a.depth = c.d_depth.p + (int64_t)p0 * g.kp_cap;
    a.status = c.d_status.p + (int64_t)p0 * g.kp_cap;
    a.match_r = c.d_match.p + (int64_t)p0 * g.kp_cap;
    a.out_stride = g.kp_cap;
    a.lkpR = c.d_lvl_kp.p + (i0 + 1) * g.lvl_kp_cap;
    a.lkp_stride = 2 * (int64_t)g.lvl_kp_cap;
    a.lcntR = c.d_lvl_count.p + (i0 + 1) * g.nlevels;
    a.lcnt_stride = 2 * (int64_t)g.nlevels;
    stereo_buffers(c, a, p0);
    stereo_consts(bf, fx, a);
    return a;
}

// Pairs [p0, p0 + n) of the extracted batch at d_in; buckets_built: extract_range's k_orb launch built them.
void stereo_range(orbfe_ctx& c, const uint8_t* d_in, int64_t pitch, int p0, int n, double bf, float fx,
                  hipStream_t s, bool buckets_built = false) {
    const StereoArgs a = stereo_args(c, d_in, pitch, p0, bf, fx);
    HIPCK(launch_stereo(c.geo, a, n, s, buckets_built));
}

// Marks the end of a batch enqueue on s: orbfe_batch_pack_device orders its k_pack after it, whatever
// stream the caller packs on.
// A batch enqueue only notes that its results are pending on last_stream; the event is recorded when a call
// on another stream needs them (wait_batch_done).  Recording it at every enqueue put a marker packet between a
// handle's consecutive chains: with two handles on two queues it delayed the next chain's first kernel by
// ~6 us (8-pair step 0.162 -> 0.159 ms with one handle, tools/small_batch.py).
void record_batch_done(orbfe_ctx& c, hipStream_t s) {
    (void)s;
    c.batch_done_rec = true;
}

// order `caller` after the handle's last batch (a no-op on the batch's own stream)
void wait_batch_done(orbfe_ctx& c, hipStream_t caller) {
    if (!c.batch_done_rec || caller == c.last_stream) return;
    if (!c.batch_done) HIPCK(hipEventCreateWithFlags(&c.batch_done, hipEventDisableTiming));
    HIPCK(hipEventRecord(c.batch_done, c.last_stream));
    HIPCK(hipStreamWaitEvent(caller, c.batch_done, 0));
}

void enqueue_stereo_batch(orbfe_ctx& c, int n_pairs, double bf, float fx, hipStream_t s) {
    if (n_pairs <= 0) return;
    if (2 * n_pairs > c.last_images) throw Error(ORBFE_ESTATE, "stereo batch needs 2*n_pairs extracted images");
    stereo_range(c, c.last_in, c.last_pitch, 0, n_pairs, bf, fx, s);
    c.last_bf = bf;
    c.last_fx = fx;
    prof_mark(c, s, 5);
    if (c.prof_on && c.prof_n < c.prof_max) ++c.prof_n;
    c.last_pairs = n_pairs;
    record_batch_done(c, s);
}

constexpr size_t kMaxGraphs = 8;  // cached executable graphs per handle (e.g. two double-buffered inputs)

uint64_t bits_of(double v) { uint64_t b; std::memcpy(&b, &v, 8); return b; }
uint64_t bits_of(float v) { uint32_t b; std::memcpy(&b, &v, 4); return b; }
uint64_t bits_of(const void* p) { return (uint64_t)(uintptr_t)p; }

// Runs enqueue(stream) on s: directly, or (graphs on) as the executable graph cached under key — captured
// on the first use of the key, replayed with one hipGraphLaunch afterwards.  Every pointer and argument
// the enqueue bakes into its launches must be part of the key (c.gen stands for the handle's buffers).
template <class F>
void run_enqueue(orbfe_ctx& c, int kind, std::vector<uint64_t> key, hipStream_t s, F&& enqueue) {
    if (!(c.graph_mask & kind) || c.prof_on) {
        enqueue(s);
        return;
    }
    key.push_back(c.gen);
    for (orbfe_ctx::GraphEntry& e : c.graphs)
        if (e.key == key) {
            HIPCK(hipGraphLaunch(e.exec, s));
            HIPCK(hipEventRecord(e.done, s));
            ++c.graph_launches;
            return;
        }
    if (!c.cap_stream) HIPCK(hipStreamCreateWithFlags(&c.cap_stream, hipStreamNonBlocking));
    hipGraph_t gr = nullptr;
    HIPCK(hipStreamBeginCapture(c.cap_stream, hipStreamCaptureModeThreadLocal));
    try {
        enqueue(c.cap_stream);
    } catch (...) {
        if (hipStreamEndCapture(c.cap_stream, &gr) == hipSuccess && gr) (void)hipGraphDestroy(gr);
        throw;
    }
    HIPCK(hipStreamEndCapture(c.cap_stream, &gr));
    hipGraphExec_t ex = nullptr;
    const hipError_t e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    HIPCK(e);
    hipEvent_t done = nullptr;
    if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
        (void)hipGraphExecDestroy(ex);
        throw Error(ORBFE_EHIP, "hipEventCreateWithFlags failed");
    }
    if (c.graphs.size() >= kMaxGraphs) {
        orbfe_ctx::retire(c.graphs.front());
        c.graphs.erase(c.graphs.begin());
    }
    c.graphs.push_back({std::move(key), ex, done});
    ++c.graph_captures;
    HIPCK(hipGraphLaunch(ex, s));
    HIPCK(hipEventRecord(done, s));
    ++c.graph_launches;
}

// The whole front-end for n_pairs pairs as up to kLanes concurrent chunks, each on its own internal
// stream (fork from / join into the caller's stream with events): the latency-bound stages of one chunk
// overlap the issue-bound stages of another.  Chunk 0 carries the profiling marks.
void enqueue_frontend(orbfe_ctx& c, const uint8_t* d_in, int64_t pitch, int n_pairs, double bf, float fx,
                      hipStream_t s) {
    if (n_pairs <= 0) return;
    check_extract(c, pitch, 2 * n_pairs);
    const int K = std::max(1, std::min(c.lanes, n_pairs));
    if (K == 1) {
        prepare_pyramid(c, 2 * n_pairs);
        run_enqueue(c, ORBFE_GRAPH_BATCH, {1, bits_of(d_in), (uint64_t)pitch, (uint64_t)n_pairs, bits_of(bf), bits_of(fx)}, s,
                    [&](hipStream_t q) {
                        const bool fuse = orb_fuses_bucket(c.geo);
                        const StereoArgs sa = stereo_args(c, d_in, pitch, 0, bf, fx);
                        extract_range(c, d_in, pitch, 0, 2 * n_pairs, q, true, -1, true, fuse ? &sa : nullptr);
                        stereo_range(c, d_in, pitch, 0, n_pairs, bf, fx, q, fuse);
                        prof_mark(c, q, 5);
                    });
    } else {
        // the lane streams, events and each chunk's pyramid tables exist before a graph capture starts
        if (!c.lane_stream[0]) {
            for (int k = 0; k < kLanes; ++k) {
                HIPCK(hipStreamCreateWithFlags(&c.lane_stream[k], hipStreamNonBlocking));
                HIPCK(hipEventCreateWithFlags(&c.lane_done[k], hipEventDisableTiming));
            }
            HIPCK(hipEventCreateWithFlags(&c.lane_fork, hipEventDisableTiming));
        }
        auto chunk = [&](int k, int& p0, int& p1) {
            p0 = (int)((int64_t)n_pairs * k / K);
            p1 = (int)((int64_t)n_pairs * (k + 1) / K);
        };
        for (int k = 0; k < K; ++k) {
            int p0, p1;
            chunk(k, p0, p1);
            prepare_pyramid(c, 2 * (p1 - p0));
        }
        // fork / join with events; under ORBFE_GRAPH_BATCH the whole fork / join is captured as ONE graph with
        // K parallel branches (the lane streams join the capture through the fork event)
        run_enqueue(c, ORBFE_GRAPH_BATCH,
                    {2, bits_of(d_in), (uint64_t)pitch, (uint64_t)n_pairs, bits_of(bf), bits_of(fx), (uint64_t)K}, s,
                    [&](hipStream_t q) {
                        HIPCK(hipMemsetAsync(c.d_overflow.p, 0, sizeof(int), q));
                        HIPCK(hipEventRecord(c.lane_fork, q));
                        for (int k = 0; k < K; ++k) {
                            int p0, p1;
                            chunk(k, p0, p1);
                            hipStream_t ls = c.lane_stream[k];
                            HIPCK(hipStreamWaitEvent(ls, c.lane_fork, 0));
                            const bool fuse = orb_fuses_bucket(c.geo);
                            const StereoArgs sa = stereo_args(c, d_in, pitch, p0, bf, fx);
                            extract_range(c, d_in, pitch, 2 * p0, 2 * (p1 - p0), ls, k == 0, k, false,
                                          fuse ? &sa : nullptr);
                            stereo_range(c, d_in, pitch, p0, p1 - p0, bf, fx, ls, fuse);
                            if (k == 0) prof_mark(c, ls, 5);
                            HIPCK(hipEventRecord(c.lane_done[k], ls));
                        }
                        for (int k = 0; k < K; ++k) HIPCK(hipStreamWaitEvent(q, c.lane_done[k], 0));
                    });
    }
    if (c.prof_on && c.prof_n < c.prof_max) ++c.prof_n;
    c.last_in = d_in;
    c.last_pitch = pitch;
    c.last_images = 2 * n_pairs;
    c.last_pairs = n_pairs;
    c.last_stream = s;
    c.last_bf = bf;
    c.last_fx = fx;
    record_batch_done(c, s);
}

hipStream_t own(orbfe_ctx& c) {
    if (!c.own_stream) HIPCK(hipStreamCreateWithFlags(&c.own_stream, hipStreamNonBlocking));
    return c.own_stream;
}


// Host image rows -> the pinned staging buffer (one CPU pass), then ONE contiguous host->device copy on s.
// A hipMemcpy2DAsync straight from pageable memory is staged by the runtime row by row: 6.8 ms per pair
// of 1241x376 images, against 0.4 ms for the whole pair call this way (tools/dbg/frame_extract_time.py).
// The caller synchronises s before h_in is reused.
void stage_host(orbfe_ctx& c, const uint8_t* const* imgs, int n, int width, int height, int64_t stride, int64_t pitch) {
    c.h_in.ensure((size_t)pitch * n);
    for (int i = 0; i < n; ++i) {
        uint8_t* o = c.h_in.p + (int64_t)i * pitch;
        if (stride == width) {
            std::memcpy(o, imgs[i], (size_t)width * height);
        } else {
            for (int y = 0; y < height; ++y) std::memcpy(o + (int64_t)y * width, imgs[i] + y * stride, width);
        }
    }
}

void stage_images(orbfe_ctx& c, uint8_t* dst, const uint8_t* const* imgs, int n, int width, int height,
                  int64_t stride, int64_t pitch, hipStream_t s) {
    stage_host(c, imgs, n, width, height, stride, pitch);
    HIPCK(hipMemcpyAsync(dst, c.h_in.p, (size_t)pitch * (n - 1) + (size_t)width * height, hipMemcpyHostToDevice, s));
}

void check_overflow(orbfe_ctx& c) {
    int ovf = 0;
    HIPCK(hipMemcpy(&ovf, c.d_overflow.p, sizeof(int), hipMemcpyDeviceToHost));
    if (ovf) throw Error(ORBFE_EOVERFLOW, "on-device capacity bound exceeded (code " + std::to_string(ovf) + ")");
}

}  // namespace

// ============================================================================================ C ABI
extern "C" {

const char* orbfe_last_error(void) { return g_err.c_str(); }

const char* orbfe_version(void) { return "orbfe 0.1 gfx950 (HIP, wave64, integer/bitwise, no MFMA)"; }

int32_t orbfe_abi_version(void) { return ORBFE_ABI_VERSION; }

int orbfe_create(const orbfe_params* params, orbfe_handle* out) {
    return guarded([&] {
        if (!params || !out) throw Error(ORBFE_EINVAL, "null argument");
        std::unique_ptr<orbfe_ctx> c(new orbfe_ctx());
        c->prm = *params;
        build_tables(*c);
        *out = c.release();
    });
}

int orbfe_destroy(orbfe_handle h) {
    return guarded([&] {
        if (h && h->last_stream) (void)hipStreamSynchronize(h->last_stream);
        delete h;
    });
}

int orbfe_get_scales(orbfe_handle h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                     int32_t* n_per_level) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        for (int l = 0; l < h->prm.nlevels; ++l) {
            if (scale) scale[l] = h->sf[l];
            if (inv_scale) inv_scale[l] = h->isf[l];
            if (sigma2) sigma2[l] = h->s2[l];
            if (inv_sigma2) inv_sigma2[l] = h->is2[l];
            if (n_per_level) n_per_level[l] = h->n_per_level[l];
        }
    });
}

int orbfe_batch_reserve(orbfe_handle h, int32_t width, int32_t height, int32_t max_images) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        reserve(*h, width, height, max_images);
    });
}

int orbfe_extract(orbfe_handle h, const uint8_t* img, int32_t width, int32_t height, int32_t stride,
                  orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        *n_out = 0;
        invalidate_results(*h);
        if (width <= 0 || height <= 0) return;  // _image.empty() -> return (ORBextractor.cpp:1045-1046)
        if (!img || stride < width) throw Error(ORBFE_EINVAL, "bad image pointer / stride");
        reserve(*h, width, height, std::max(h->max_images, 1));
        hipStream_t s = own(*h);
        const size_t bytes = (size_t)width * height;
        h->d_in.ensure(bytes);
        stage_images(*h, h->d_in.p, &img, 1, width, height, stride, (int64_t)bytes, s);
        enqueue_extract(*h, h->d_in.p, (int64_t)bytes, 1, s);
        int n = 0;
        HIPCK(hipMemcpyAsync(&n, h->d_count.p, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
        check_overflow(*h);
        h->have_single = true;
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "keypoint buffer too small");
        if (n > 0) {
            if (kps) HIPCK(hipMemcpy(kps, h->d_kps.p, (size_t)n * sizeof(orbfe_keypoint), hipMemcpyDeviceToHost));
            if (desc) HIPCK(hipMemcpy(desc, h->d_desc.p, (size_t)n * 32, hipMemcpyDeviceToHost));
        }
    });
}

int orbfe_pyramid(orbfe_handle h, int32_t level, uint8_t* out, int32_t sheared, int32_t* w_out, int32_t* h_out) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (!h->have_single) throw Error(ORBFE_ESTATE, "no image extracted with orbfe_extract yet");
        if (level < 0 || level >= h->geo.nlevels) throw Error(ORBFE_EINVAL, "level out of range");
        const LevelGeo& L = h->geo.lv[level];
        if (w_out) *w_out = L.w;
        if (h_out) *h_out = L.h;
        if (!out) return;
        if (!sheared) {
            const uint8_t* src = level == 0 ? h->d_in.p : h->d_ws.p + L.ws_off;
            const size_t spitch = level == 0 ? (size_t)L.w : (size_t)L.pitch;
            HIPCK(hipMemcpy2D(out, L.w, src, spitch, L.w, L.h, hipMemcpyDeviceToHost));
            return;
        }
        // the reference caster's stride-ignoring view, built on the device (k_shear)
        hipStream_t s = own(*h);
        h->d_shear.ensure((size_t)h->geo.shear_bytes);
        HIPCK(launch_shear(h->geo, h->d_in.p, (int64_t)h->W * h->H, h->d_ws.p, h->d_shear.p, 1, s));
        HIPCK(hipMemcpyAsync(out, h->d_shear.p + L.shear_off, (size_t)L.w * L.h, hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
    });
}

int orbfe_frame_extract(orbfe_handle h, const uint8_t* left, const uint8_t* right, int32_t width, int32_t height,
                        int32_t stride, double bf, float fx, int32_t want_pyramid) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        invalidate_results(*h);
        const bool empty = width <= 0 || height <= 0;  // operator_kd: _image.empty() -> return (:1045-1046)
        if (!empty) {
            if (!left || !right || stride < width) throw Error(ORBFE_EINVAL, "bad image pointer / stride");
            reserve(*h, width, height, std::max(h->max_images, 2));
        }
        const Geo& g = h->geo;
        const size_t cap = empty ? 0 : (size_t)g.kp_cap;
        size_t o = 0;
        auto take = [&](size_t bytes) { const size_t r = o; o = (o + bytes + 255) & ~(size_t)255; return r; };
        h->fo_ovf = take(sizeof(int));
        h->fo_count = take(2 * sizeof(int));
        h->fo_kps = take(2 * cap * sizeof(orbfe_keypoint));
        h->fo_desc = take(2 * cap * 32);
        h->fo_uR = take(cap * sizeof(float));
        h->fo_depth = take(cap * sizeof(float));
        h->fo_status = take(cap);
        h->fo_match = take(cap * sizeof(int32_t));
        h->fo_shear = take(empty ? 0 : 2 * (size_t)g.shear_bytes);
        h->h_frame.ensure(o);
        uint8_t* hb = h->h_frame.p;
        if (empty) {
            std::memset(hb + h->fo_count, 0, 2 * sizeof(int));
            std::memset(hb + h->fo_ovf, 0, sizeof(int));
            h->have_frame = true;
            return;
        }
        if (want_pyramid < 0 || want_pyramid > 2) throw Error(ORBFE_EINVAL, "want_pyramid must be 0, 1 or 2");
        const bool lazy = want_pyramid == 2;
        if (lazy) want_pyramid = 0;  // the views go to the ring below, not into the frame buffer
        hipStream_t s = own(*h);
        const int64_t pitch = ((int64_t)width * height + 255) & ~(int64_t)255;
        h->d_in.ensure(2 * (size_t)pitch);
        if (want_pyramid) h->d_shear.ensure(2 * (size_t)g.shear_bytes);
        if (lazy) {
            const uint8_t* before = h->d_ring.p;
            h->d_ring.ensure((size_t)kFrameRing * 2 * (size_t)g.shear_bytes);
            if (h->d_ring.p != before)
                for (int64_t& r : h->ring_serial) r = 0;
        }
        const uint8_t* pair[2] = {left, right};
        stage_host(*h, pair, 2, width, height, stride, pitch);
        uint8_t* hb_dev = nullptr;  // the frame buffer as the device addresses it (k_copy_segments writes it)
        HIPCK(hipHostGetDevicePointer((void**)&hb_dev, hb, 0));
        // everything after the host copy is one enqueue (a graph replay when graphs are on): both images in,
        // the 2-image pipeline, stereo, optionally the sheared views, every result out to pinned memory
        const std::vector<uint64_t> key = {2, bits_of(h->h_in.p), bits_of(h->d_in.p), bits_of(hb),
                                           bits_of(want_pyramid ? h->d_shear.p : nullptr), (uint64_t)width,
                                           (uint64_t)height, bits_of(bf), bits_of(fx), (uint64_t)o};
        prepare_pyramid(*h, 2);
        run_enqueue(*h, ORBFE_GRAPH_FRAME, key, s, [&](hipStream_t q) {
            HIPCK(hipMemcpyAsync(h->d_in.p, h->h_in.p, (size_t)pitch + (size_t)width * height, hipMemcpyHostToDevice, q));
            const bool fuse = orb_fuses_bucket(g);
            const StereoArgs sa = stereo_args(*h, h->d_in.p, pitch, 0, bf, fx);
            extract_range(*h, h->d_in.p, pitch, 0, 2, q, false, -1, true, fuse ? &sa : nullptr);
            stereo_range(*h, h->d_in.p, pitch, 0, 1, bf, fx, q, fuse);
            if (want_pyramid) HIPCK(launch_shear(g, h->d_in.p, pitch, h->d_ws.p, h->d_shear.p, 2, q));
            // every result into the page-locked frame buffer with ONE kernel's stores over PCIe (k_copy_segments;
            // 8-9 copy-engine transfers cost ~60 us per frame in fixed costs, rocprof round 4)
            CopySegs cp{};
            auto seg = [&](size_t off, const void* src, size_t bytes) {
                cp.seg[cp.n++] = {(const uint32_t*)src, (uint32_t*)(hb_dev + off), (uint32_t)((bytes + 3) / 4)};
            };
            seg(h->fo_ovf, h->d_overflow.p, sizeof(int));
            seg(h->fo_count, h->d_count.p, 2 * sizeof(int));
            seg(h->fo_kps, h->d_kps.p, 2 * cap * sizeof(orbfe_keypoint));
            seg(h->fo_desc, h->d_desc.p, 2 * cap * 32);
            seg(h->fo_uR, h->d_uR.p, cap * sizeof(float));
            seg(h->fo_depth, h->d_depth.p, cap * sizeof(float));
            seg(h->fo_status, h->d_status.p, cap);
            seg(h->fo_match, h->d_match.p, cap * sizeof(int32_t));
            if (want_pyramid) seg(h->fo_shear, h->d_shear.p, 2 * (size_t)g.shear_bytes);
            HIPCK(launch_copy_segments(cp, q));
        });
        const int64_t serial = ++h->frame_serial;
        h->ring_serial[serial % kFrameRing] = 0;
        if (lazy) {  // both views into this serial's ring slot, behind the graph (one graph for every slot)
            HIPCK(launch_shear(g, h->d_in.p, pitch, h->d_ws.p,
                               h->d_ring.p + (size_t)(serial % kFrameRing) * 2 * (size_t)g.shear_bytes, 2, s));
            h->ring_serial[serial % kFrameRing] = serial;
        }
        h->frame_ring = lazy;
        HIPCK(hipStreamSynchronize(s));
        h->last_in = h->d_in.p;
        h->last_pitch = h->frame_pitch = pitch;
        h->last_images = 2;
        h->last_pairs = 1;
        h->last_stream = s;
        h->last_bf = bf;
        h->last_fx = fx;
        int ovf = 0;
        std::memcpy(&ovf, hb + h->fo_ovf, sizeof(int));
        if (ovf) throw Error(ORBFE_EOVERFLOW, "on-device capacity bound exceeded (code " + std::to_string(ovf) + ")");
        h->have_frame = true;
        h->frame_pyr = want_pyramid != 0;
    });
}

int orbfe_frame_fetch(orbfe_handle h, int32_t side, orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (!h->have_frame) throw Error(ORBFE_ESTATE, "no frame extracted with orbfe_frame_extract");
        if (side != 0 && side != 1) throw Error(ORBFE_EINVAL, "side must be 0 (left) or 1 (right)");
        const uint8_t* hb = h->h_frame.p;
        int n = 0;
        std::memcpy(&n, hb + h->fo_count + side * sizeof(int), sizeof(int));
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "keypoint buffer too small");
        const size_t kc = (size_t)h->geo.kp_cap;
        if (n && kps) std::memcpy(kps, hb + h->fo_kps + side * kc * sizeof(orbfe_keypoint), n * sizeof(orbfe_keypoint));
        if (n && desc) std::memcpy(desc, hb + h->fo_desc + side * kc * 32, (size_t)n * 32);
    });
}

int orbfe_frame_fetch_stereo(orbfe_handle h, float* u_right, float* depth, int8_t* status, int32_t* match_r,
                             int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (!h->have_frame) throw Error(ORBFE_ESTATE, "no frame extracted with orbfe_frame_extract");
        const uint8_t* hb = h->h_frame.p;
        int n = 0;
        std::memcpy(&n, hb + h->fo_count, sizeof(int));
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "buffer too small");
        if (n && u_right) std::memcpy(u_right, hb + h->fo_uR, n * sizeof(float));
        if (n && depth) std::memcpy(depth, hb + h->fo_depth, n * sizeof(float));
        if (n && status) std::memcpy(status, hb + h->fo_status, n);
        if (n && match_r) std::memcpy(match_r, hb + h->fo_match, n * sizeof(int32_t));
    });
}

int orbfe_frame_pyramid(orbfe_handle h, int32_t side, int32_t level, uint8_t* out, int32_t* w_out, int32_t* h_out) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (!h->have_frame || h->W <= 0 || h->last_images != 2) throw Error(ORBFE_ESTATE, "no frame extracted");
        if (side != 0 && side != 1) throw Error(ORBFE_EINVAL, "side must be 0 (left) or 1 (right)");
        if (level < 0 || level >= h->geo.nlevels) throw Error(ORBFE_EINVAL, "level out of range");
        const Geo& g = h->geo;
        const LevelGeo& L = g.lv[level];
        if (w_out) *w_out = L.w;
        if (h_out) *h_out = L.h;
        if (!out) return;
        if (!h->frame_pyr) {  // not requested at extraction: build (or take from the ring) and fetch both views now
            hipStream_t s = own(*h);
            const uint8_t* src;
            if (h->frame_ring) {
                src = h->d_ring.p + (size_t)(h->frame_serial % kFrameRing) * 2 * (size_t)g.shear_bytes;
            } else {
                h->d_shear.ensure(2 * (size_t)g.shear_bytes);
                HIPCK(launch_shear(g, h->d_in.p, h->frame_pitch, h->d_ws.p, h->d_shear.p, 2, s));
                src = h->d_shear.p;
            }
            HIPCK(hipMemcpyAsync(h->h_frame.p + h->fo_shear, src, 2 * (size_t)g.shear_bytes, hipMemcpyDeviceToHost, s));
            HIPCK(hipStreamSynchronize(s));
            h->frame_pyr = true;
        }
        std::memcpy(out, h->h_frame.p + h->fo_shear + side * (size_t)g.shear_bytes + L.shear_off, (size_t)L.w * L.h);
    });
}

int orbfe_frame_serial(orbfe_handle h, int64_t* serial, int64_t* oldest) {
    return guarded([&] {
        if (!h || !serial) throw Error(ORBFE_EINVAL, "null argument");
        *serial = h->frame_serial;
        if (oldest) *oldest = std::max<int64_t>(1, h->frame_serial - kFrameRing + 1);
    });
}

int orbfe_frame_pyramid_fetch(orbfe_handle h, int64_t serial, int32_t side, uint8_t* out, int64_t bytes) {
    return guarded([&] {
        if (!h || !out) throw Error(ORBFE_EINVAL, "null argument");
        if (side != 0 && side != 1) throw Error(ORBFE_EINVAL, "side must be 0 (left) or 1 (right)");
        const Geo& g = h->geo;
        if (bytes != g.shear_bytes) throw Error(ORBFE_EINVAL, "out must hold the frame geometry's shear_bytes");
        if (serial < 1 || h->ring_serial[serial % kFrameRing] != serial)
            throw Error(ORBFE_ESTATE, "that frame's pyramid has left the device ring (fetch it before " +
                                          std::to_string(kFrameRing) + " newer frames)");
        hipStream_t s = own(*h);
        HIPCK(hipMemcpyAsync(out, h->d_ring.p + ((size_t)(serial % kFrameRing) * 2 + side) * (size_t)g.shear_bytes,
                             (size_t)g.shear_bytes, hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
    });
}

int orbfe_undistort_points(orbfe_handle h, const float* K4, const float* dist, int32_t n_dist, const float* xy, int32_t n,
                           int32_t stride, float* out) {
    return guarded([&] {
        if (!h || !K4 || !dist || (n > 0 && (!xy || !out))) throw Error(ORBFE_EINVAL, "null argument");
        if (n < 0 || stride < 2) throw Error(ORBFE_EINVAL, "bad point count / stride");
        if (n_dist != 4 && n_dist != 5) throw Error(ORBFE_EINVAL, "distortion must be (k1, k2, p1, p2[, k3])");
        if (n == 0) return;
        UndistortArgs a{K4[0], K4[1], K4[2], K4[3], dist[0], dist[1], dist[2], dist[3], n_dist == 5 ? dist[4] : 0.f};
        hipStream_t s = own(*h);
        h->d_uin.ensure((size_t)n * stride);
        h->d_uout.ensure((size_t)n * 2);
        HIPCK(hipMemcpyAsync(h->d_uin.p, xy, (size_t)n * stride * sizeof(float), hipMemcpyHostToDevice, s));
        HIPCK(launch_undistort(h->d_uin.p, n, stride, h->d_uout.p, a, s));
        HIPCK(hipMemcpyAsync(out, h->d_uout.p, (size_t)n * 2 * sizeof(float), hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
    });
}

int orbfe_stereo_match(orbfe_handle hl, orbfe_handle hr, double bf, float fx, float* u_right, float* depth,
                       int8_t* status, int32_t* match_r, int32_t n_left) {
    return guarded([&] {
        if (!hl || !hr) throw Error(ORBFE_EINVAL, "null handle");
        if (!hl->have_single || !hr->have_single) throw Error(ORBFE_ESTATE, "both handles must have extracted");
        if (hl->W != hr->W || hl->H != hr->H || hl->prm.nlevels != hr->prm.nlevels)
            throw Error(ORBFE_EINVAL, "left/right extractors differ in geometry");
        const Geo& g = hl->geo;
        StereoArgs a{};
        a.kpsL = hl->d_kps.p;
        a.kpsR = hr->d_kps.p;
        a.descL = hl->d_desc.p;
        a.descR = hr->d_desc.p;
        a.countL = hl->d_count.p;
        a.countR = hr->d_count.p;
        a.lvl0L = hl->d_in.p;
        a.lvl0R = hr->d_in.p;
        a.wsL = hl->d_ws.p;
        a.wsR = hr->d_ws.p;
        a.u_right = hl->d_uR.p;
        a.depth = hl->d_depth.p;
        a.status = hl->d_status.p;
        a.match_r = hl->d_match.p;
        a.out_stride = g.kp_cap;
        a.lkpR = hr->d_lvl_kp.p;
        a.lcntR = hr->d_lvl_count.p;
        stereo_buffers(*hl, a, 0);
        a.kp_stride = 0;
        stereo_consts(bf, fx, a);
        hipStream_t s = own(*hl);
        HIPCK(launch_stereo(g, a, 1, s));
        int nL = 0;
        HIPCK(hipMemcpyAsync(&nL, hl->d_count.p, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
        if (n_left != nL) throw Error(ORBFE_EINVAL, "n_left does not match the left keypoint count");
        if (nL == 0) return;
        if (u_right) HIPCK(hipMemcpy(u_right, hl->d_uR.p, nL * sizeof(float), hipMemcpyDeviceToHost));
        if (depth) HIPCK(hipMemcpy(depth, hl->d_depth.p, nL * sizeof(float), hipMemcpyDeviceToHost));
        if (status) HIPCK(hipMemcpy(status, hl->d_status.p, nL, hipMemcpyDeviceToHost));
        if (match_r) HIPCK(hipMemcpy(match_r, hl->d_match.p, nL * sizeof(int32_t), hipMemcpyDeviceToHost));
    });
}

int orbfe_extract_batch_device(orbfe_handle h, const uint8_t* d_images, int64_t img_pitch, int32_t n_images,
                               void* hip_stream) {
    return guarded([&] {
        if (!h || !d_images) throw Error(ORBFE_EINVAL, "null argument");
        if (h->W <= 0) throw Error(ORBFE_ESTATE, "call orbfe_batch_reserve first");
        invalidate_results(*h);
        enqueue_extract(*h, d_images, img_pitch, n_images, (hipStream_t)hip_stream);
    });
}

int orbfe_stereo_batch_device(orbfe_handle h, int32_t n_pairs, double bf, float fx, void* hip_stream) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        invalidate_results(*h);  // overwrites the stereo buffers and the row buckets
        enqueue_stereo_batch(*h, n_pairs, bf, fx, (hipStream_t)hip_stream);
    });
}

int orbfe_frontend_batch_device(orbfe_handle h, const uint8_t* d_images, int64_t img_pitch, int32_t n_pairs,
                                double bf, float fx, void* hip_stream) {
    return guarded([&] {
        if (!h || !d_images) throw Error(ORBFE_EINVAL, "null argument");
        if (h->W <= 0) throw Error(ORBFE_ESTATE, "call orbfe_batch_reserve first");
        invalidate_results(*h);
        enqueue_frontend(*h, d_images, img_pitch, n_pairs, bf, fx, (hipStream_t)hip_stream);
    });
}

int orbfe_set_lanes(orbfe_handle h, int32_t lanes) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (lanes < 1 || lanes > kLanes) throw Error(ORBFE_EINVAL, "lanes must be 1..4");
        h->lanes = lanes;
    });
}

int orbfe_batch_view_get(orbfe_handle h, orbfe_batch_view* v) {
    return guarded([&] {
        if (!h || !v) throw Error(ORBFE_EINVAL, "null argument");
        v->kp_cap = h->geo.kp_cap;
        v->n_images = h->last_images;
        v->n_pairs = h->last_pairs;
        v->kps = h->d_kps.p;
        v->desc = h->d_desc.p;
        v->count = h->d_count.p;
        v->u_right = h->d_uR.p;
        v->depth = h->d_depth.p;
        v->status = h->d_status.p;
        v->match_r = h->d_match.p;
        v->overflow = h->d_overflow.p;
    });
}

int orbfe_batch_status(orbfe_handle h, int32_t* overflow) {
    return guarded([&] {
        if (!h || !overflow) throw Error(ORBFE_EINVAL, "null argument");
        if (h->last_stream) HIPCK(hipStreamSynchronize(h->last_stream));
        int ovf = 0;
        if (h->d_overflow.p) HIPCK(hipMemcpy(&ovf, h->d_overflow.p, sizeof(int), hipMemcpyDeviceToHost));
        *overflow = ovf;
    });
}

int64_t record_bytes(int kp_cap) {
    const int64_t raw = 8 + 2 * (int64_t)kp_cap * (int64_t)sizeof(orbfe_keypoint) + 2 * (int64_t)kp_cap * 32 +
                        (int64_t)kp_cap * 9;
    return (raw + 15) / 16 * 16;
}

int orbfe_batch_record_bytes(orbfe_handle h, int64_t* bytes) {
    return guarded([&] {
        if (!h || !bytes) throw Error(ORBFE_EINVAL, "null argument");
        if (h->W <= 0) throw Error(ORBFE_ESTATE, "call orbfe_batch_reserve first");
        *bytes = record_bytes(h->geo.kp_cap);
    });
}

int orbfe_batch_pack_device(orbfe_handle h, uint8_t* d_records, int64_t rec_bytes, int32_t pair0, int32_t n_pairs,
                            void* hip_stream) {
    return guarded([&] {
        if (!h || !d_records) throw Error(ORBFE_EINVAL, "null argument");
        if (pair0 < 0 || n_pairs < 0 || pair0 + n_pairs > h->last_pairs)
            throw Error(ORBFE_EINVAL, "pair range outside the last stereo batch");
        if (rec_bytes != record_bytes(h->geo.kp_cap)) throw Error(ORBFE_EINVAL, "record size does not match kp_cap");
        if (reinterpret_cast<uintptr_t>(d_records) & 3) throw Error(ORBFE_EINVAL, "records must be 4-byte aligned");
        // device memory, or page-locked host memory the device can address (k_pack then writes the records over
        // PCIe straight into host memory); pageable host memory is refused instead of faulting on the device
        hipPointerAttribute_t pa{};
        if (hipPointerGetAttributes(&pa, d_records) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(ORBFE_EINVAL, "records buffer is neither device memory nor registered host memory");
        }
        if (pa.type == hipMemoryTypeHost) {
            if (!pa.devicePointer) throw Error(ORBFE_EINVAL, "host records buffer is not mapped for the device");
            d_records = (uint8_t*)pa.devicePointer;
        } else if (pa.type != hipMemoryTypeDevice && pa.type != hipMemoryTypeManaged) {
            throw Error(ORBFE_EINVAL, "records buffer is neither device memory nor registered host memory");
        }
        PackArgs a{h->d_count.p, h->d_kps.p, h->d_desc.p, h->d_uR.p, h->d_depth.p, h->d_status.p, h->geo.kp_cap,
                   rec_bytes};
        // the records are read after the batch that produced them, on whichever stream the caller packs
        wait_batch_done(*h, (hipStream_t)hip_stream);
        HIPCK(launch_pack(a, d_records, pair0, n_pairs, (hipStream_t)hip_stream));
    });
}

int64_t compact_record_bytes(int kp_cap) { return (8 + 91 * (int64_t)kp_cap + 15) / 16 * 16; }

int orbfe_batch_compact_record_bytes(orbfe_handle h, int64_t* bytes) {
    return guarded([&] {
        if (!h || !bytes) throw Error(ORBFE_EINVAL, "null argument");
        if (h->W <= 0) throw Error(ORBFE_ESTATE, "call orbfe_batch_reserve first");
        *bytes = compact_record_bytes(h->geo.kp_cap);
    });
}

int orbfe_batch_pack_compact_device(orbfe_handle h, uint8_t* d_records, int64_t rec_bytes, int32_t pair0,
                                    int32_t n_pairs, void* hip_stream) {
    return guarded([&] {
        if (!h || !d_records) throw Error(ORBFE_EINVAL, "null argument");
        if (pair0 < 0 || n_pairs < 0 || pair0 + n_pairs > h->last_pairs)
            throw Error(ORBFE_EINVAL, "pair range outside the last stereo batch");
        if (rec_bytes != compact_record_bytes(h->geo.kp_cap))
            throw Error(ORBFE_EINVAL, "record size does not match kp_cap");
        if (reinterpret_cast<uintptr_t>(d_records) & 3) throw Error(ORBFE_EINVAL, "records must be 4-byte aligned");
        for (int l = 0; l < h->geo.nlevels; ++l)  // the compact format's 14-bit level coordinates (k_pack_compact)
            if (h->geo.lv[l].w > (1 << kCompactXYBits) || h->geo.lv[l].h > (1 << kCompactXYBits))
                throw Error(ORBFE_EINVAL, "compact records hold level coordinates below 16384 px only");
        hipPointerAttribute_t pa{};
        if (hipPointerGetAttributes(&pa, d_records) != hipSuccess || pa.type != hipMemoryTypeDevice) {
            (void)hipGetLastError();
            throw Error(ORBFE_EINVAL, "compact records must be device memory");
        }
        PackArgs a{h->d_count.p, h->d_kps.p, h->d_desc.p, h->d_uR.p, h->d_depth.p, h->d_status.p, h->geo.kp_cap,
                   rec_bytes};
        CompactScales sc{};
        for (int l = 0; l < kMaxLevels; ++l) sc.inv_scale[l] = l < h->geo.nlevels ? h->geo.inv_scale[l] : 1.f;
        wait_batch_done(*h, (hipStream_t)hip_stream);
        HIPCK(launch_pack_compact(a, sc, d_records, pair0, n_pairs, (hipStream_t)hip_stream));
    });
}

int orbfe_batch_fetch(orbfe_handle h, int32_t image, orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (image < 0 || image >= h->last_images) throw Error(ORBFE_EINVAL, "image index out of range");
        if (h->last_stream) HIPCK(hipStreamSynchronize(h->last_stream));
        check_overflow(*h);
        int n = 0;
        HIPCK(hipMemcpy(&n, h->d_count.p + image, sizeof(int), hipMemcpyDeviceToHost));
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "keypoint buffer too small");
        const size_t o = (size_t)image * h->geo.kp_cap;
        if (n && kps) HIPCK(hipMemcpy(kps, h->d_kps.p + o, n * sizeof(orbfe_keypoint), hipMemcpyDeviceToHost));
        if (n && desc) HIPCK(hipMemcpy(desc, h->d_desc.p + o * 32, (size_t)n * 32, hipMemcpyDeviceToHost));
    });
}

int orbfe_batch_fetch_stereo(orbfe_handle h, int32_t pair, float* u_right, float* depth, int8_t* status,
                             int32_t* match_r, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (pair < 0 || pair >= h->last_pairs) throw Error(ORBFE_EINVAL, "pair index out of range");
        if (h->last_stream) HIPCK(hipStreamSynchronize(h->last_stream));
        check_overflow(*h);
        int n = 0;
        HIPCK(hipMemcpy(&n, h->d_count.p + 2 * pair, sizeof(int), hipMemcpyDeviceToHost));
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "buffer too small");
        const size_t o = (size_t)pair * h->geo.kp_cap;
        if (n && u_right) HIPCK(hipMemcpy(u_right, h->d_uR.p + o, n * sizeof(float), hipMemcpyDeviceToHost));
        if (n && depth) HIPCK(hipMemcpy(depth, h->d_depth.p + o, n * sizeof(float), hipMemcpyDeviceToHost));
        if (n && status) HIPCK(hipMemcpy(status, h->d_status.p + o, n, hipMemcpyDeviceToHost));
        if (n && match_r) HIPCK(hipMemcpy(match_r, h->d_match.p + o, n * sizeof(int32_t), hipMemcpyDeviceToHost));
    });
}

int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b, int32_t* out) {
    return guarded([&] {
        if (!a || !b || !out) throw Error(ORBFE_EINVAL, "null argument");
        uint64_t x[4], y[4];
        std::memcpy(x, a, 32);
        std::memcpy(y, b, 32);
        *out = __builtin_popcountll(x[0] ^ y[0]) + __builtin_popcountll(x[1] ^ y[1]) + __builtin_popcountll(x[2] ^ y[2]) +
               __builtin_popcountll(x[3] ^ y[3]);
    });
}

int orbfe_grid_query(const int32_t* cell_off, const int32_t* cell_idx, int32_t cols, int32_t rows, const double* kp_x,
                     const double* kp_y, const int32_t* kp_oct, int32_t n_kp, const double* frame4, int32_t n_q,
                     const double* qx, const double* qy, const double* qr, const int32_t* qmin, const int32_t* qmax,
                     int32_t* out_off, int32_t* out_idx, int64_t cap) {
    return guarded([&] {
        if (!cell_off || !frame4 || (n_q > 0 && (!qx || !qy || !qr || !qmin || !qmax || !out_off)))
            throw Error(ORBFE_EINVAL, "null argument");
        if (cols <= 0 || rows <= 0 || n_q < 0 || n_kp < 0) throw Error(ORBFE_EINVAL, "bad sizes");
        const double minX = frame4[0], minY = frame4[1], invW = frame4[2], invH = frame4[3];
        int64_t n = 0;
        out_off[0] = 0;
        for (int q = 0; q < n_q; ++q) {
            const double x = qx[q], y = qy[q], r = qr[q];
            const int lo = qmin[q], hi = qmax[q];
            // Frame.get_features_in_area (Frame.py:373-416) in the Python floats' double arithmetic; int()
            // truncates toward zero like the C conversion
            const int x0 = std::max(0, (int)((x - minX - r) * invW));
            const int x1 = std::min(cols - 1, (int)((x - minX + r) * invW));
            const int y0 = std::max(0, (int)((y - minY - r) * invH));
            const int y1 = std::min(rows - 1, (int)((y - minY + r) * invH));
            if (x0 < cols && x1 >= 0 && y0 < rows && y1 >= 0) {
                const bool check = lo > 0 || hi >= 0;
                for (int ix = x0; ix <= x1; ++ix)
                    for (int iy = y0; iy <= y1; ++iy) {
                        const int c = ix * rows + iy;
                        for (int k = cell_off[c]; k < cell_off[c + 1]; ++k) {
                            const int g = cell_idx[k];
                            if (g < 0 || g >= n_kp) throw Error(ORBFE_EINVAL, "grid index out of range");
                            if (check) {
                                if (kp_oct[g] < lo) continue;
                                if (hi >= 0 && kp_oct[g] > hi) continue;
                            }
                            if (std::fabs(kp_x[g] - x) < r && std::fabs(kp_y[g] - y) < r) {
                                if (n < cap) out_idx[n] = g;
                                ++n;
                            }
                        }
                    }
            }
            if (n > INT32_MAX) throw Error(ORBFE_ECAPACITY, "too many candidates");
            out_off[q + 1] = (int32_t)n;
        }
        if (n > cap) throw Error(ORBFE_ECAPACITY, "candidate buffer too small (out_off[n_q] holds the need)");
    });
}

// The sequential candidate selection of the two tracking searches over precomputed distances, in double
// (this file is built with -ffp-contract=off: `u - mbf * invzc` stays two roundings like Python's).
// blocked[i] = "slot i holds a map point with observations" (the `if mvpMapPoints[i]: if ...observations()
// > 0: continue` test); a match stores the query's own flag there, as the reference's assignment changes
// what later queries of the same search read.
namespace {
void check_select(int32_t n_q, const int32_t* off, const int32_t* idx, const int32_t* dist, const double* u_right,
                  const uint8_t* blocked, int32_t n_frame, const int32_t* best_idx) {
    if (n_q < 0 || n_frame < 0) throw Error(ORBFE_EINVAL, "negative size");
    if (n_q > 0 && (!off || !best_idx)) throw Error(ORBFE_EINVAL, "null argument");
    if (n_q > 0 && off[n_q] > 0 && (!idx || !dist || !u_right || !blocked)) throw Error(ORBFE_EINVAL, "null argument");
    for (int32_t k = 0; n_q > 0 && k < off[n_q]; ++k)
        if (idx[k] < 0 || idx[k] >= n_frame) throw Error(ORBFE_EINVAL, "candidate index out of range");
}
}  // namespace

int orbfe_select_f_f(int32_t n_q, const int32_t* off, const int32_t* idx, const int32_t* dist, const double* u,
                     const double* invzc, const double* radius, const uint8_t* q_obs, const double* u_right,
                     uint8_t* blocked, int32_t n_frame, double mbf, int32_t th_high, int32_t* best_idx) {
    return guarded([&] {
        check_select(n_q, off, idx, dist, u_right, blocked, n_frame, best_idx);
        for (int32_t q = 0; q < n_q; ++q) {
            int best_dist = 256, best = -1;
            for (int32_t k = off[q]; k < off[q + 1]; ++k) {  // ORBMatcher.py:348-368
                const int i2 = idx[k];
                if (blocked[i2]) continue;
                if (u_right[i2] > 0) {
                    const double ur = u[q] - mbf * invzc[q];
                    if (std::fabs(ur - u_right[i2]) > radius[q]) continue;
                }
                if (dist[k] < best_dist) {
                    best_dist = dist[k];
                    best = i2;
                }
            }
            if (best_dist <= th_high) {  // :370-372
                best_idx[q] = best;
                blocked[best] = q_obs[q];
            } else {
                best_idx[q] = -1;
            }
        }
    });
}

int orbfe_select_f_p(int32_t n_q, const int32_t* off, const int32_t* idx, const int32_t* dist, const double* xr,
                     const double* r_scaled, const int32_t* kp_octave, const uint8_t* q_obs, const double* u_right,
                     uint8_t* blocked, int32_t n_frame, double nnratio, int32_t th_high, int32_t* best_idx) {
    return guarded([&] {
        check_select(n_q, off, idx, dist, u_right, blocked, n_frame, best_idx);
        for (int32_t q = 0; q < n_q; ++q) {
            int bd = 256, bl = -1, bd2 = 256, bl2 = -1, bi = -1;
            for (int32_t k = off[q]; k < off[q + 1]; ++k) {  // ORBMatcher.py:246-275
                const int i = idx[k];
                if (blocked[i]) continue;
                if (u_right[i] > 0 && std::fabs(xr[q] - u_right[i]) > r_scaled[q]) continue;
                const int d = dist[k];
                if (d < bd) {
                    bd2 = bd;
                    bd = d;
                    bl2 = bl;
                    bl = kp_octave[i];
                    bi = i;
                } else if (d < bd2) {
                    bl2 = kp_octave[i];
                    bd2 = d;
                }
            }
            best_idx[q] = -1;
            if (bd <= th_high && !(bl == bl2 && (double)bd > nnratio * (double)bd2)) {  // :276-281
                best_idx[q] = bi;
                blocked[bi] = q_obs[q];
            }
        }
    });
}

int orbfe_hamming_matrix(orbfe_handle h, const uint8_t* a_desc, int32_t n_a, const uint8_t* b_desc, int32_t n_b,
                         int32_t* out) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (n_a < 0 || n_b < 0) throw Error(ORBFE_EINVAL, "negative size");
        if (n_a == 0 || n_b == 0) return;
        std::lock_guard<std::mutex> lk(h->hmu);
        hipStream_t s = own(*h);
        h->d_hq.ensure((size_t)n_a * 32);
        h->d_ht.ensure((size_t)n_b * 32);
        h->d_hres.ensure((size_t)n_a * n_b);
        HIPCK(hipMemcpyAsync(h->d_hq.p, a_desc, (size_t)n_a * 32, hipMemcpyHostToDevice, s));
        HIPCK(hipMemcpyAsync(h->d_ht.p, b_desc, (size_t)n_b * 32, hipMemcpyHostToDevice, s));
        HIPCK(launch_hamming_matrix(h->d_hq.p, n_a, h->d_ht.p, n_b, h->d_hres.p, s));
        HIPCK(hipMemcpyAsync(out, h->d_hres.p, (size_t)n_a * n_b * sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCK(hipStreamSynchronize(s));
    });
}

namespace {
// shared body of orbfe_hamming_search / orbfe_hamming_csr
void hamming_run(orbfe_ctx& c, const uint8_t* q, int nq, const uint8_t* t, int nt, const int32_t* off,
                 const int32_t* idx, std::vector<int>* top2, int32_t* all_d) {
    if (nq < 0 || nt < 0) throw Error(ORBFE_EINVAL, "negative size");
    if (nq == 0) return;
    if (off[0] != 0) throw Error(ORBFE_EINVAL, "cand_off[0] must be 0");
    for (int i = 0; i < nq; ++i)
        if (off[i + 1] < off[i]) throw Error(ORBFE_EINVAL, "cand_off must be non-decreasing");
    const int ncand = off[nq];
    for (int i = 0; i < ncand; ++i)
        if (idx[i] < 0 || idx[i] >= nt) throw Error(ORBFE_EINVAL, "candidate index out of range");
    std::lock_guard<std::mutex> lk(c.hmu);
    hipStream_t s = own(c);
    c.d_hq.ensure((size_t)nq * 32);
    c.d_ht.ensure((size_t)std::max(nt, 1) * 32);
    c.d_hoff.ensure((size_t)nq + 1);
    c.d_hidx.ensure((size_t)std::max(ncand, 1));
    c.d_hres.ensure((size_t)4 * nq + std::max(ncand, 1));
    HIPCK(hipMemcpyAsync(c.d_hq.p, q, (size_t)nq * 32, hipMemcpyHostToDevice, s));
    if (nt) HIPCK(hipMemcpyAsync(c.d_ht.p, t, (size_t)nt * 32, hipMemcpyHostToDevice, s));
    HIPCK(hipMemcpyAsync(c.d_hoff.p, off, ((size_t)nq + 1) * sizeof(int), hipMemcpyHostToDevice, s));
    if (ncand) HIPCK(hipMemcpyAsync(c.d_hidx.p, idx, (size_t)ncand * sizeof(int), hipMemcpyHostToDevice, s));
    int* r = c.d_hres.p;
    int* dall = all_d ? r + 4 * nq : nullptr;
    HIPCK(launch_hamming_search(c.d_hq.p, nq, c.d_ht.p, c.d_hoff.p, c.d_hidx.p, r, r + nq, r + 2 * nq, r + 3 * nq, dall,
                                s));
    if (top2) {
        top2->resize((size_t)4 * nq);
        HIPCK(hipMemcpyAsync(top2->data(), r, top2->size() * sizeof(int), hipMemcpyDeviceToHost, s));
    }
    if (all_d && ncand) HIPCK(hipMemcpyAsync(all_d, dall, (size_t)ncand * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCK(hipStreamSynchronize(s));
}
}  // namespace

int orbfe_hamming_search(orbfe_handle h, const uint8_t* query_desc, int32_t n_query, const uint8_t* train_desc,
                         int32_t n_train, const int32_t* cand_off, const int32_t* cand_idx, int32_t* best_dist,
                         int32_t* best_idx, int32_t* second_dist, int32_t* second_idx) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        std::vector<int> res;
        hamming_run(*h, query_desc, n_query, train_desc, n_train, cand_off, cand_idx, &res, nullptr);
        for (int i = 0; i < n_query; ++i) {
            if (best_dist) best_dist[i] = res[i];
            if (best_idx) best_idx[i] = res[n_query + i];
            if (second_dist) second_dist[i] = res[2 * n_query + i];
            if (second_idx) second_idx[i] = res[3 * n_query + i];
        }
    });
}

int orbfe_hamming_csr(orbfe_handle h, const uint8_t* query_desc, int32_t n_query, const uint8_t* train_desc,
                      int32_t n_train, const int32_t* cand_off, const int32_t* cand_idx, int32_t* out_dist) {
    return guarded([&] {
        if (!h || !out_dist) throw Error(ORBFE_EINVAL, "null argument");
        hamming_run(*h, query_desc, n_query, train_desc, n_train, cand_off, cand_idx, nullptr, out_dist);
    });
}

int orbfe_profile_begin(orbfe_handle h, int32_t max_batches) {
    return guarded([&] {
        if (!h || max_batches < 0) throw Error(ORBFE_EINVAL, "bad argument");
        const size_t need = (size_t)max_batches * kProfEvents;
        while (h->prof_ev.size() < need) {
            hipEvent_t e;
            HIPCK(hipEventCreate(&e));
            h->prof_ev.push_back(e);
        }
        h->prof_max = max_batches;
        h->prof_n = 0;
        h->prof_on = max_batches > 0;
    });
}

int orbfe_profile_read(orbfe_handle h, float* ms_per_stage, int32_t* n_batches) {
    return guarded([&] {
        if (!h || !ms_per_stage) throw Error(ORBFE_EINVAL, "null argument");
        for (int k = 0; k < ORBFE_NSTAGES; ++k) ms_per_stage[k] = 0.f;
        for (int b = 0; b < h->prof_n; ++b) {
            hipEvent_t* e = &h->prof_ev[(size_t)b * kProfEvents];
            HIPCK(hipEventSynchronize(e[ORBFE_NSTAGES]));
            for (int k = 0; k < ORBFE_NSTAGES; ++k) {
                float ms = 0.f;
                HIPCK(hipEventElapsedTime(&ms, e[k], e[k + 1]));
                ms_per_stage[k] += ms;
            }
        }
        if (n_batches) *n_batches = h->prof_n;
        h->prof_on = false;
    });
}

int orbfe_microbench(orbfe_handle h, int32_t stage, int32_t variant, int32_t reps, float* ms) {
    return guarded([&] {
        if (!h || !ms || reps <= 0) throw Error(ORBFE_EINVAL, "bad argument");
        if (h->last_images <= 0 || !h->last_in) throw Error(ORBFE_ESTATE, "run a batch first");
        const Geo& g = h->geo;
        const int n = h->last_images;
        hipStream_t s = h->last_stream;
        hipEvent_t e0, e1;
        HIPCK(hipEventCreate(&e0));
        HIPCK(hipEventCreate(&e1));
        auto run = [&] {
            switch (stage) {
                case 0:
                    // variant 6: the one-launch cascade with the automatic strip count for this batch, 100 + S:
                    // with S strips (tools/microbench.py); 7: the per-level launches whatever the batch size
                    if (variant == 6 || variant >= 100) {
                        orbfe_ctx::Cascade* cs = nullptr;
                        for (int S = variant >= 100 ? variant - 100 : cascade_strips(*h, n); S > 0; S += 4) {
                            if (!(cs = find_cascade(*h, S))) {
                                std::unique_ptr<orbfe_ctx::Cascade> ns = resize_strips(*h, S);
                                if (ns) h->cascades.push_back(std::move(ns));
                                cs = find_cascade(*h, S);
                            }
                            if (cs || S > g.lv[g.nlevels - 1].h) break;
                        }
                        if (!cs) throw Error(ORBFE_EINVAL, "no cascade strip count fits the LDS");
                        HIPCK(launch_resize_cascade(g, h->last_in, h->last_pitch, h->d_ws.p, h->d_xt.p, h->d_yt.p,
                                                    cs->tab.p, cs->S, cs->off_b, cs->off_x, cs->lds, n, s));
                        break;
                    }
                    for (int l = 1; l < g.nlevels; ++l)
                        HIPCK(launch_resize(g, l, h->last_in, h->last_pitch, h->d_ws.p, h->d_xt.p, h->d_yt.p, n, s,
                                            variant == 7 ? 0 : variant));
                    break;
                case 1:
                    HIPCK(launch_detect(g, h->d_cells.p, h->last_in, h->last_pitch, h->d_ws.p, h->d_cell_count.p,
                                        h->d_slots.p, n, s, variant));
                    break;
                case 2:
                    HIPCK(launch_octree(g, h->d_cells.p, h->d_cell_count.p, h->d_slots.p, h->d_octab.p, h->d_kd.p,
                                        h->d_kn.p, h->d_lvl_kp.p, h->d_lvl_count.p, h->d_overflow.p, h->maxcell, n, s,
                                        variant));
                    break;
                case 3:
                    // variant 0: k_orb (production), 8: 8-wave workgroups, 12 / 9 / 10: 2 / 4 / 16 keypoints per
                    // wave (the round-1 unfused k_blur + k_describe pair is in the git history, round 1)
                    HIPCK(launch_orb(g, h->last_in, h->last_pitch, h->d_ws.p, h->d_lvl_kp.p, h->d_lvl_count.p,
                                     h->d_kps.p, h->d_desc.p, h->d_count.p, n, h->d_orb.p, s, variant == 12 ? 2 : variant));
                    break;
                case 4:
                    if (h->last_pairs <= 0) throw Error(ORBFE_ESTATE, "no stereo batch");
                    enqueue_stereo_batch(*h, h->last_pairs, h->last_bf, h->last_fx, s);
                    break;
                case 5:
                    // the HBM writes a blurred pyramid would add (every level of every image, w x h bytes each):
                    // the lower bound of its cost in any design that writes one
                    h->d_shear.ensure((size_t)n * (size_t)g.shear_bytes);
                    HIPCK(hipMemsetD8Async((hipDeviceptr_t)h->d_shear.p, 0x5A, (size_t)n * (size_t)g.shear_bytes, s));
                    break;
                default:
                    throw Error(ORBFE_EINVAL, "bad stage");
            }
        };
        run();  // warm
        HIPCK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) run();
        HIPCK(hipEventRecord(e1, s));
        HIPCK(hipEventSynchronize(e1));
        float t = 0.f;
        HIPCK(hipEventElapsedTime(&t, e0, e1));
        *ms = t / reps;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    });
}

int orbfe_debug_candidates(orbfe_handle h, int32_t level, int32_t* xyr, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (!h->have_single) throw Error(ORBFE_ESTATE, "no image extracted with orbfe_extract yet");
        if (level < 0 || level >= h->geo.nlevels) throw Error(ORBFE_EINVAL, "level out of range");
        const LevelGeo& L = h->geo.lv[level];
        std::vector<int> cnt(std::max(L.ncell, 1));
        std::vector<uint32_t> slots(h->geo.slot_total);
        if (L.ncell)
            HIPCK(hipMemcpy(cnt.data(), h->d_cell_count.p + L.cell0, L.ncell * sizeof(int), hipMemcpyDeviceToHost));
        HIPCK(hipMemcpy(slots.data(), h->d_slots.p, slots.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        int n = 0;
        for (int i = 0; i < L.ncell; ++i) {
            const CellGeo& cg = h->cells[L.cell0 + i];
            for (int j = 0; j < cnt[i]; ++j, ++n) {
                if (n >= cap) continue;
                const uint32_t k = slots[cg.slot_off + j];
                xyr[3 * n] = (int)((k & 0xFFFFFFu) % (uint32_t)L.w) - kBorder;
                xyr[3 * n + 1] = (int)((k & 0xFFFFFFu) / (uint32_t)L.w) - kBorder;
                xyr[3 * n + 2] = (int)(k >> 24);
            }
        }
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "buffer too small");
    });
}

int orbfe_debug_selected(orbfe_handle h, int32_t level, int32_t* xyr, int32_t cap, int32_t* n_out) {
    return guarded([&] {
        if (!h || !n_out) throw Error(ORBFE_EINVAL, "null argument");
        if (!h->have_single) throw Error(ORBFE_ESTATE, "no image extracted with orbfe_extract yet");
        if (level < 0 || level >= h->geo.nlevels) throw Error(ORBFE_EINVAL, "level out of range");
        const LevelGeo& L = h->geo.lv[level];
        int n = 0;
        HIPCK(hipMemcpy(&n, h->d_lvl_count.p + level, sizeof(int), hipMemcpyDeviceToHost));
        std::vector<uint32_t> kp(std::max(n, 1));
        if (n) HIPCK(hipMemcpy(kp.data(), h->d_lvl_kp.p + L.kp_off, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        *n_out = n;
        if (n > cap) throw Error(ORBFE_ECAPACITY, "buffer too small");
        for (int i = 0; i < n; ++i) {
            xyr[3 * i] = (int)((kp[i] & 0xFFFFFFu) % (uint32_t)L.w) - kBorder;
            xyr[3 * i + 1] = (int)((kp[i] & 0xFFFFFFu) / (uint32_t)L.w) - kBorder;
            xyr[3 * i + 2] = (int)(kp[i] >> 24);
        }
    });
}

int orbfe_set_graphs(orbfe_handle h, int32_t mask) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (mask & ~(ORBFE_GRAPH_FRAME | ORBFE_GRAPH_BATCH)) throw Error(ORBFE_EINVAL, "unknown graph flags");
        h->graph_mask = mask;
        h->drop_graphs();
    });
}

int orbfe_graph_stats(orbfe_handle h, int64_t* captures, int64_t* launches, int32_t* cached) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (captures) *captures = h->graph_captures;
        if (launches) *launches = h->graph_launches;
        if (cached) *cached = (int32_t)h->graphs.size();
    });
}

int orbfe_set_octree_kernel(orbfe_handle h, int32_t kernel) {
    return guarded([&] {
        if (!h) throw Error(ORBFE_EINVAL, "null handle");
        if (kernel != 0 && kernel != 1) throw Error(ORBFE_EINVAL, "kernel must be 0 (automatic) or 1 (per-candidate)");
        h->octree_force = kernel == 1;
        if (h->W > 0) {  // re-derive the reserved geometry's choice (build_geometry's rule)
            invalidate_results(*h);
            h->drop_graphs();
            Geo& g = h->geo;
            g.oct_v = h->octree_force || octree_bins_lds_bytes(g, h->maxcell) > 150 * 1024 ? 1 : 0;
            prepare_kernels(*h);
        }
    });
}

int orbfe_get_octree_kernel(orbfe_handle h, int32_t* kernel, int64_t* bins_lds_bytes) {
    return guarded([&] {
        if (!h || !kernel) throw Error(ORBFE_EINVAL, "null argument");
        if (h->W <= 0) throw Error(ORBFE_ESTATE, "no geometry reserved yet");
        *kernel = h->geo.oct_v;
        if (bins_lds_bytes) *bins_lds_bytes = (int64_t)octree_bins_lds_bytes(h->geo, h->maxcell);
    });
}

int orbfe_debug_detect_stats(orbfe_handle h, int64_t* stats) {
    return guarded([&] {
        if (!h || !stats) throw Error(ORBFE_EINVAL, "null argument");
        if (h->last_images <= 0 || !h->last_in) throw Error(ORBFE_ESTATE, "run a batch first");
        const Geo& g = h->geo;
        DevBuf<int> d;
        d.ensure(4);
        HIPCK(hipMemset(d.p, 0, 4 * sizeof(int)));
        if (g.ncells > 0)
            HIPCK(launch_detect(g, h->d_cells.p, h->last_in, h->last_pitch, h->d_ws.p, h->d_cell_count.p, h->d_slots.p,
                                h->last_images, h->last_stream, 0, d.p));
        HIPCK(hipStreamSynchronize(h->last_stream));
        int v[4];
        HIPCK(hipMemcpy(v, d.p, sizeof(v), hipMemcpyDeviceToHost));
        for (int k = 0; k < 3; ++k) stats[k] = v[k];
    });
}

int orbfe_debug_cascade_profile(orbfe_handle h, int64_t* marks, int64_t n_marks, int32_t* n_strips) {
    return guarded([&] {
        if (!h || !marks || !n_strips) throw Error(ORBFE_EINVAL, "null argument");
        if (h->last_images <= 0 || !h->last_in) throw Error(ORBFE_ESTATE, "run a batch first");
        const Geo& g = h->geo;
        const int n = h->last_images;
        int S = cascade_strips(*h, n);
        orbfe_ctx::Cascade* cs = nullptr;
        while (S > 0 && !(cs = find_cascade(*h, S)) && S <= g.lv[g.nlevels - 1].h) S += 4;
        if (!cs) throw Error(ORBFE_ESTATE, "the last batch did not take the cascade");
        const int64_t need = (int64_t)n * cs->S * 32;
        *n_strips = cs->S;
        if (n_marks < need) throw Error(ORBFE_ECAPACITY, "buffer too small (32 marks per image and strip)");
        DevBuf<long long> d;
        d.ensure(need);
        HIPCK(hipMemset(d.p, 0, need * sizeof(long long)));
        HIPCK(launch_resize_cascade(g, h->last_in, h->last_pitch, h->d_ws.p, h->d_xt.p, h->d_yt.p, cs->tab.p, cs->S,
                                    cs->off_b, cs->off_x, cs->lds, n, h->last_stream, nullptr, d.p));
        HIPCK(hipStreamSynchronize(h->last_stream));
        HIPCK(hipMemcpy(marks, d.p, need * sizeof(long long), hipMemcpyDeviceToHost));
    });
}

int orbfe_debug_octree_profile(orbfe_handle h, int64_t* marks, int64_t n) {
    return guarded([&] {
        if (!h || !marks) throw Error(ORBFE_EINVAL, "null argument");
        if (h->last_images <= 0 || !h->last_in) throw Error(ORBFE_ESTATE, "run a batch first");
        const Geo& g = h->geo;
        const int64_t need = (int64_t)h->last_images * g.nlevels * 64;
        if (n < need) throw Error(ORBFE_ECAPACITY, "buffer too small");
        DevBuf<long long> d;
        d.ensure(need);
        HIPCK(hipMemset(d.p, 0, need * sizeof(long long)));
        HIPCK(launch_octree(g, h->d_cells.p, h->d_cell_count.p, h->d_slots.p, h->d_octab.p, h->d_kd.p, h->d_kn.p,
                            h->d_lvl_kp.p, h->d_lvl_count.p, h->d_overflow.p, h->maxcell, h->last_images, h->last_stream,
                            0, d.p));
        HIPCK(hipStreamSynchronize(h->last_stream));
        HIPCK(hipMemcpy(marks, d.p, need * sizeof(long long), hipMemcpyDeviceToHost));
    });
}

}  // extern "C"
