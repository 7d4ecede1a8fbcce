/*
 * orb_oracle.cpp — TEST INFRASTRUCTURE ONLY: the CPU checker for the gfx950 extractor.
 *
 * A restatement (not a copy) of the reference ORB-SLAM2 extractor in
 * /root/reference/pyORBExtractor/ORBextractor.cpp and of the OpenCV 4.x pixel primitives it calls
 * (cv::resize INTER_LINEAR, cv::FAST 9/16 + NMS, cv::GaussianBlur 7x7 fixed point, cv::fastAtan2,
 * cvRound).  Each function cites the reference lines it follows.
 *
 * PARITY: UNPINNED for the extractor (OpenCV is absent from the image, so the reference extractor
 * cannot be compiled, and the reference ships no extractor outputs).  The orchestration follows the
 * reference line by line; the OpenCV primitives follow SURVEY.md Appendix A.
 *
 * Floating point: built with -ffp-contract=off.  The two descriptor sample-coordinate expressions are
 * written with explicit fmaf() because the reference build (-O3 -march=native, CMakeLists.txt:12-13)
 * contracts them so on FMA hosts (verified with GCC 11 on a probe of the same expression shape).
 * (float)cos / sin of a float are glibc's sinf/cosf (ARM optimized-routines algorithm, x86-64
 * FMA ifunc variant of glibc 2.35) restated below and checked exhaustively against the host libm.
 *
 * Octree tie-break: DistributeOctTree sorts (size, ExtractorNode*) pairs (ORBextractor.cpp:683), so
 * equal-size nodes are ordered by heap address.  The canonical order used here (and on the GPU) is
 * node creation order — what any monotonic allocator yields.
 */
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <list>
#include <utility>
#include <vector>

namespace {

constexpr int kPatchSize = 31;     // ORBextractor.cpp:72
constexpr int kHalfPatch = 15;     // :73
constexpr int kEdge = 19;          // :74
constexpr int kCoefBits = 11;      // INTER_RESIZE_COEF_BITS
constexpr int kCoefScale = 1 << kCoefBits;

const int8_t kPattern[1024] = {
#include "../pyorbslam_amd/csrc/brief_pattern.inc"
};

// ---------------------------------------------------------------- rounding helpers (cvRound etc.)
inline int round_even_f(float v) { return (int)std::lrintf(v); }   // cvRound(float): half to even
inline int round_even_d(double v) { return (int)std::lrint(v); }   // cvRound(double)
inline int floor_f(float v) { int i = (int)v; return i - (i > v); } // cvFloor(float)
inline int ceil_f(float v) { int i = (int)v; return i + (i < v); }  // cvCeil(float)
inline short sat_short(int v) { return (short)std::min(std::max(v, -32768), 32767); }
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

// ---------------------------------------------------------------- glibc sinf / cosf (FMA variant)
struct SinCosTab { double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4; };
const SinCosTab kSC[2] = {
    {{1, -1, -1, 1}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p+0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1, -1, -1, 1}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p+0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};

inline float sc_sin_poly(double x, double x2, const SinCosTab& t) {
    double x3 = x * x2, s1 = std::fma(x2, t.s3, t.s2), x5 = x2 * x3, s = std::fma(x3, t.s1, x);
    return (float)std::fma(x5, s1, s);
}
inline float sc_cos_poly(double x2, const SinCosTab& t) {
    double x4 = x2 * x2, c1 = std::fma(x2, t.c1, t.c0), c2 = std::fma(x2, t.c4, t.c3), x6 = x2 * x4;
    double c = std::fma(x4, t.c2, c1);
    return (float)std::fma(x6, c2, c);
}
inline unsigned top12(float y) { uint32_t u; std::memcpy(&u, &y, 4); return (u >> 20) & 0x7ff; }

// Only the |y| < 120 range is restated (descriptor angles are in [0, 2*pi)).
float glibc_cosf(float y) {
    unsigned t = top12(y);
    double x = y;
    if (t <= 0x3f3) return t <= 0x397 ? 1.0f : sc_cos_poly(x * x, kSC[0]);
    double r = x * kSC[0].hpi_inv;
    int n = (((int)r) + 0x800000) >> 24;
    x = std::fma(-(double)n, kSC[0].hpi, x);
    const SinCosTab& p = (n & 2) ? kSC[1] : kSC[0];
    if (n & 1) return sc_sin_poly(x * kSC[0].sign[n & 3], x * x, p);
    return sc_cos_poly(x * x, p);
}
float glibc_sinf(float y) {
    unsigned t = top12(y);
    double x = y;
    if (t <= 0x3f3) return t <= 0x397 ? y : sc_sin_poly(x, x * x, kSC[0]);
    double r = x * kSC[0].hpi_inv;
    int n = (((int)r) + 0x800000) >> 24;
    x = std::fma(-(double)n, kSC[0].hpi, x);
    const SinCosTab& p = (n & 2) ? kSC[1] : kSC[0];
    if ((n & 1) == 0) return sc_sin_poly(x * kSC[0].sign[n & 3], x * x, p);
    return sc_cos_poly(x * x, p);
}

// ---------------------------------------------------------------- cv::fastAtan2 (degrees)
const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::fabs(x), ay = std::fabs(y), a;
    if (ax >= ay) {
        float c = ay / (ax + (float)DBL_EPSILON), c2 = c * c;
        a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    } else {
        float c = ax / (ay + (float)DBL_EPSILON), c2 = c * c;
        a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------------------------- extractor configuration
struct Config {
    int nfeatures, nlevels, iniTh, minTh, simd;
    double scaleFactor;  // ORBextractor.h:101 keeps the (float) ctor argument in a double
    std::vector<float> sf, isf, s2, is2;
    std::vector<int> nPerLevel;
    int umax[kHalfPatch + 1];
};

// ORBextractor.cpp:410-470
bool make_config(const orbfe_params* p, Config& C) {
    if (!p || p->nlevels < 1 || p->nlevels > 32 || p->nfeatures < 0 || !(p->scale_factor > 0)) return false;
    C.nfeatures = p->nfeatures;
    C.nlevels = p->nlevels;
    C.iniTh = p->ini_th_fast;
    C.minTh = p->min_th_fast;
    C.simd = p->resize_simd_lanes;
    C.scaleFactor = (double)p->scale_factor;
    const int L = C.nlevels;
    C.sf.assign(L, 1.0f);
    C.s2.assign(L, 1.0f);
    for (int i = 1; i < L; ++i) {
        C.sf[i] = (float)((double)C.sf[i - 1] * C.scaleFactor);
        C.s2[i] = C.sf[i] * C.sf[i];
    }
    C.isf.resize(L);
    C.is2.resize(L);
    for (int i = 0; i < L; ++i) {
        C.isf[i] = 1.0f / C.sf[i];
        C.is2[i] = 1.0f / C.s2[i];
    }
    C.nPerLevel.assign(L, 0);
    const float factor = (float)(1.0 / C.scaleFactor);
    float want = C.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; ++l) {
        C.nPerLevel[l] = round_even_f(want);
        sum += C.nPerLevel[l];
        want *= factor;
    }
    C.nPerLevel[L - 1] = std::max(C.nfeatures - sum, 0);

    // intensity-centroid disk: row half-widths, made symmetric (ORBextractor.cpp:454-469)
    const int vmax = floor_f(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = ceil_f(kHalfPatch * std::sqrt(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) C.umax[v] = round_even_d(std::sqrt(hp2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (C.umax[v0] == C.umax[v0 + 1]) ++v0;
        C.umax[v] = v0;
        ++v0;
    }
    return true;
}

struct Image {
    int w = 0, h = 0;
    std::vector<uint8_t> px;  // tight, stride == w
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// ---------------------------------------------------------------- cv::resize INTER_AREA fast path, 8U
// cv::resize switches INTER_LINEAR with an exact 2x step (|scale - 2| < DBL_EPSILON both ways) to INTER_AREA,
// whose fast path (resizeAreaFast_Invoker + ResizeAreaFastVec_SIMD_8u, OpenCV 4.x imgproc/resize.cpp) averages
// every 2 x 2 block: the vector loop (u16 lanes = simd / 2 per step, while dx <= w - lanes) stores
// v_rshr_pack_store<2>, i.e. (a + b + c + d + 2) >> 2; the scalar tail saturate_cast<uchar>(sum * 0.25f), i.e.
// sum / 4 rounded half to even.  Parity unpinned (OpenCV is absent), like the linear path.
void resize_area2(const uint8_t* src, int sw, int sstride, uint8_t* dst, int dw, int dh, int simd) {
    (void)sw;
    const int lanes = simd / 2;
    const int xv = lanes > 0 ? dw / lanes * lanes : 0;
    for (int dy = 0; dy < dh; ++dy) {
        const uint8_t* S0 = src + (size_t)(2 * dy) * sstride;
        const uint8_t* S1 = S0 + sstride;
        for (int dx = 0; dx < dw; ++dx) {
            const int sum = S0[2 * dx] + S0[2 * dx + 1] + S1[2 * dx] + S1[2 * dx + 1];
            dst[(size_t)dy * dw + dx] = dx < xv ? (uint8_t)((sum + 2) >> 2) : sat_u8(round_even_f((float)sum * 0.25f));
        }
    }
}

// ---------------------------------------------------------------- cv::resize INTER_LINEAR, 8U
void resize_linear(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh, int simd) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    {
        const int isx = (int)std::lrint(scale_x), isy = (int)std::lrint(scale_y);
        if (std::fabs(scale_x - isx) < DBL_EPSILON && std::fabs(scale_y - isy) < DBL_EPSILON && isx == 2 && isy == 2) {
            resize_area2(src, sw, sstride, dst, dw, dh, simd);
            return;
        }
    }
    std::vector<int> xofs(dw);
    std::vector<short> ax(2 * dw);
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
        xofs[dx] = sx;
        ax[2 * dx] = sat_short(round_even_f((1.f - fx) * kCoefScale));
        ax[2 * dx + 1] = sat_short(round_even_f(fx * kCoefScale));
    }
    // end of the span OpenCV's VResizeLinearVec_32s8u covers (16-lane / 8-lane steps)
    int xv = 0;
    if (simd > 0) {
        while (xv <= dw - simd) xv += simd;
        while (xv < dw - simd / 2) xv += simd / 2;
    }
    std::vector<int> H0(dw), H1(dw);
    auto hrow = [&](int sy, std::vector<int>& H) {
        const uint8_t* S = src + (size_t)sy * sstride;
        for (int dx = 0; dx < dw; ++dx) {
            const int sx = xofs[dx];
            H[dx] = dx < xmax ? S[sx] * ax[2 * dx] + S[sx + 1] * ax[2 * dx + 1] : S[sx] * kCoefScale;
        }
    };
    auto clip = [](int v, int n) { return v >= 0 ? (v < n ? v : n - 1) : 0; };
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = floor_f(fy);
        fy -= sy;
        const int b0 = sat_short(round_even_f((1.f - fy) * kCoefScale));
        const int b1 = sat_short(round_even_f(fy * kCoefScale));
        hrow(clip(sy, sh), H0);
        hrow(clip(sy + 1, sh), H1);
        uint8_t* D = dst + (size_t)dy * dw;
        for (int x = 0; x < dw; ++x) {
            if (x < xv) {
                // v_mul_hi(v_pack(S>>4), beta) summed, v_rshr_pack_u<2>
                const int a0 = std::min(H0[x] >> 4, 32767), a1 = std::min(H1[x] >> 4, 32767);
                const int t = ((a0 * b0) >> 16) + ((a1 * b1) >> 16);
                D[x] = sat_u8((t + 2) >> 2);
            } else {
                D[x] = sat_u8((H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
}

// ---------------------------------------------------------------- cv::FAST 9/16 with NMS
// circle offsets (dx, dy) in OpenCV's order
const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// segment test: 9 contiguous circle pixels all darker than v-t or all brighter than v+t
bool segment_test(const uint8_t* p, const int* off, int t) {
    const int v = p[0];
    for (int pol = 0; pol < 2; ++pol) {
        int run = 0;
        for (int k = 0; k < 25; ++k) {
            const int x = p[off[k & 15]];
            const bool hit = pol == 0 ? x < v - t : x > v + t;
            run = hit ? run + 1 : 0;
            if (run > 8) return true;
        }
    }
    return false;
}

// cornerScore: the largest threshold at which p stays a corner, i.e. max(t, M) - 1 with
// M = max over the 16 arcs of 9 of min(d) / min(-d), d_k = I(p) - I(p+o_k).
int corner_score(const uint8_t* p, const int* off, int t) {
    int d[16];
    for (int k = 0; k < 16; ++k) d[k] = (int)p[0] - (int)p[off[k]];
    int m = t;
    for (int k = 0; k < 16; ++k) {
        int lo = 255, hi = -255;
        for (int j = 0; j < 9; ++j) {
            lo = std::min(lo, d[(k + j) & 15]);
            hi = std::max(hi, d[(k + j) & 15]);
        }
        m = std::max(m, std::max(lo, -hi));
    }
    return m - 1;
}

// Detect on a w x h ROI: candidates at rows/cols 3..n-4, score map, 3x3 strict NMS in which
// anything outside the detection window (or not a corner) counts as score 0.  Output is
// row-major like OpenCV's 3-row ring buffer emits it.
int fast_roi(const uint8_t* img, int stride, int w, int h, int th, std::vector<int>& out) {
    th = std::min(std::max(th, 0), 255);
    int off[16];
    for (int k = 0; k < 16; ++k) off[k] = kCircle[k][0] + kCircle[k][1] * stride;
    std::vector<int> score((size_t)w * h, 0);
    std::vector<uint8_t> corner((size_t)w * h, 0);
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x) {
            const uint8_t* p = img + (size_t)y * stride + x;
            if (segment_test(p, off, th)) {
                corner[(size_t)y * w + x] = 1;
                score[(size_t)y * w + x] = corner_score(p, off, th);
            }
        }
    int n = 0;
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x) {
            if (!corner[(size_t)y * w + x]) continue;
            const int s = score[(size_t)y * w + x];
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (!dx && !dy) continue;
                    if (!(s > score[(size_t)(y + dy) * w + (x + dx)])) { keep = false; break; }
                }
            if (keep) {
                out.push_back(x);
                out.push_back(y);
                out.push_back(s);
                ++n;
            }
        }
    return n;
}

// ---------------------------------------------------------------- pyramid (ComputePyramid :1106-1132)
void build_pyramid(const Config& C, const uint8_t* img, int W, int H, int stride, std::vector<Image>& pyr) {
    pyr.assign(C.nlevels, Image());
    for (int l = 0; l < C.nlevels; ++l) {
        Image& L = pyr[l];
        L.w = round_even_f((float)W * C.isf[l]);
        L.h = round_even_f((float)H * C.isf[l]);
        L.px.assign((size_t)L.w * L.h, 0);
        if (l == 0) {
            for (int y = 0; y < H; ++y) std::memcpy(L.px.data() + (size_t)y * W, img + (size_t)y * stride, W);
        } else {
            const Image& P = pyr[l - 1];
            if (L.w == P.w && L.h == P.h)
                L.px = P.px;  // cv::resize copies when dsize == ssize
            else
                resize_linear(P.px.data(), P.w, P.h, P.w, L.px.data(), L.w, L.h, C.simd);
        }
    }
}

// ---------------------------------------------------------------- cells + FAST (:764-828)
struct Cand { float x, y, resp; };

void level_candidates(const Config& C, const Image& L, std::vector<Cand>& keys, int& minX, int& maxX, int& minY,
                      int& maxY) {
    const float W = 30;
    minX = kEdge - 3;
    minY = minX;
    maxX = L.w - kEdge + 3;
    maxY = L.h - kEdge + 3;
    keys.clear();
    const float width = (float)(maxX - minX), height = (float)(maxY - minY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols <= 0 || nRows <= 0) return;  // no cell loop iteration in the reference either
    const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
    std::vector<int> cell;
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
            const int y0 = (int)iniY, y1 = (int)maxYc, x0 = (int)iniX, x1 = (int)maxXc;
            const uint8_t* roi = L.row(y0) + x0;
            cell.clear();
            int n = fast_roi(roi, L.w, x1 - x0, y1 - y0, C.iniTh, cell);
            if (n == 0) n = fast_roi(roi, L.w, x1 - x0, y1 - y0, C.minTh, cell);
            for (int k = 0; k < n; ++k) {
                Cand c;
                c.x = (float)cell[3 * k] + (float)(j * wCell);
                c.y = (float)cell[3 * k + 1] + (float)(i * hCell);
                c.resp = (float)cell[3 * k + 2];
                keys.push_back(c);
            }
        }
    }
}

// ---------------------------------------------------------------- DistributeOctTree (:481-762)
struct Node {
    std::vector<int> keys;           // indices into the candidate vector, in candidate order
    int ulx = 0, uly = 0, urx = 0, bry = 0;  // UL=(ulx,uly) UR=(urx,uly) BL=(ulx,bry) BR=(urx,bry)
    bool noMore = false;
    long id = 0;                     // creation order (canonical stand-in for the node address)
    std::list<Node>::iterator self;
};

// ExtractorNode::DivideNode (:481-537)
void divide(const std::vector<Cand>& K, const Node& nd, Node c[4]) {
    const int hx = (int)std::ceil((float)(nd.urx - nd.ulx) / 2);
    const int hy = (int)std::ceil((float)(nd.bry - nd.uly) / 2);
    const int mx = nd.ulx + hx, my = nd.uly + hy;
    c[0].ulx = nd.ulx; c[0].uly = nd.uly; c[0].urx = mx; c[0].bry = my;
    c[1].ulx = mx; c[1].uly = nd.uly; c[1].urx = nd.urx; c[1].bry = my;
    c[2].ulx = nd.ulx; c[2].uly = my; c[2].urx = mx; c[2].bry = nd.bry;
    c[3].ulx = mx; c[3].uly = my; c[3].urx = nd.urx; c[3].bry = nd.bry;
    for (int k : nd.keys) {
        const Cand& kp = K[k];
        const int q = (kp.x < (float)mx ? 0 : 1) + (kp.y < (float)my ? 0 : 2);
        c[q].keys.push_back(k);
    }
    for (int q = 0; q < 4; ++q)
        if (c[q].keys.size() == 1) c[q].noMore = true;
}

// how often the reference's own output depends on heap addresses.  The careful phase sorts
// (size, ExtractorNode*) pairs (ORBextractor.cpp:683), so equal-size nodes are processed in address order:
// *  tie_runs — runs of >= 2 equal-size nodes that the careful phase divided: their processing order, and
//    so the order of their children in the list (push_front, :692-724) and of the level's keypoints, is
//    address order (here: creation order);
// *  straddle — the `>= N` break (:729-730) fell inside such a run: some of its nodes were divided and
//    others not, so WHICH keypoints the level keeps depends on the addresses.
struct TieStats {
    int straddle = 0, tie_runs = 0, careful_iters = 0;
    int run_len = 0, run_divided = 0;  // the straddled run: its equal-size nodes, how many of them were divided
};

std::vector<int> distribute(const std::vector<Cand>& K, int minX, int maxX, int minY, int maxY, int N,
                            TieStats* ts = nullptr) {
    std::vector<int> result;
    if (K.empty() || maxY - minY <= 0 || maxX - minX <= 0) return result;
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    if (nIni <= 0) return result;
    const float hX = (float)(maxX - minX) / nIni;
    long nextId = 0;
    std::list<Node> nodes;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; ++i) {
        Node n;
        n.ulx = (int)(hX * (float)i);
        n.urx = (int)(hX * (float)(i + 1));
        n.uly = 0;
        n.bry = maxY - minY;
        n.id = nextId++;
        nodes.push_back(n);
        ini[i] = &nodes.back();
    }
    for (size_t k = 0; k < K.size(); ++k) ini[(size_t)(K[k].x / hX)]->keys.push_back((int)k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) {
            it->noMore = true;
            ++it;
        } else if (it->keys.empty()) {
            it = nodes.erase(it);
        } else {
            ++it;
        }
    }
    // push the non-empty children of a divided node to the front (n1..n4), collect expandables
    typedef std::vector<std::pair<int, Node*> > Expand;
    auto push_children = [&](Node c[4], Expand& exp) {
        int added = 0;
        for (int q = 0; q < 4; ++q) {
            if (c[q].keys.empty()) continue;
            c[q].id = nextId++;
            nodes.push_front(c[q]);
            nodes.front().self = nodes.begin();
            ++added;
            if (c[q].keys.size() > 1) exp.push_back(std::make_pair((int)c[q].keys.size(), &nodes.front()));
        }
        return added;
    };
    bool finish = false;
    Expand expand;
    while (!finish) {
        const int prev = (int)nodes.size();
        expand.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->noMore) { ++it; continue; }
            Node c[4];
            divide(K, *it, c);
            push_children(c, expand);
            it = nodes.erase(it);
        }
        const int nToExpand = (int)expand.size();
        if ((int)nodes.size() >= N || (int)nodes.size() == prev) {
            finish = true;
        } else if ((int)nodes.size() + nToExpand * 3 > N) {
            while (!finish) {
                const int prevSize = (int)nodes.size();
                Expand todo = expand;
                expand.clear();
                std::sort(todo.begin(), todo.end(), [](const std::pair<int, Node*>& a, const std::pair<int, Node*>& b) {
                    return a.first != b.first ? a.first < b.first : a.second->id < b.second->id;
                });
                int jb = 0;  // the last entry divided (entries jb .. end were divided, back to front)
                bool broke = false;
                for (int j = (int)todo.size() - 1; j >= 0; --j) {
                    Node c[4];
                    divide(K, *todo[j].second, c);
                    push_children(c, expand);
                    nodes.erase(todo[j].second->self);
                    jb = j;
                    if ((int)nodes.size() >= N) { broke = true; break; }
                }
                if (ts && !todo.empty()) {
                    ++ts->careful_iters;
                    for (int j = jb; j < (int)todo.size();) {  // runs of equal size among the divided entries
                        int e = j + 1;
                        while (e < (int)todo.size() && todo[e].first == todo[j].first) ++e;
                        ts->tie_runs += e - j >= 2;
                        j = e;
                    }
                    if (broke && jb > 0 && todo[jb - 1].first == todo[jb].first) {
                        ts->straddle = 1;
                        int b = jb, e = jb;
                        while (b > 0 && todo[b - 1].first == todo[jb].first) --b;
                        while (e + 1 < (int)todo.size() && todo[e + 1].first == todo[jb].first) ++e;
                        ts->run_len = e - b + 1;
                        ts->run_divided = e - jb + 1;
                    }
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == prevSize) finish = true;
            }
        }
    }
    // keep the first maximum-response key of every node, list order (:740-759)
    for (const Node& n : nodes) {
        int best = n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (K[n.keys[k]].resp > K[best].resp) best = n.keys[k];
        result.push_back(best);
    }
    return result;
}

// ---------------------------------------------------------------- IC_Angle (:77-104)
float ic_angle(const Image& L, int cx, int cy, const int* umax) {
    int m01 = 0, m10 = 0;
    const uint8_t* c = L.row(cy) + cx;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * c[u];
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int plus = c[u + v * L.w], minus = c[u - v * L.w];
            vsum += plus - minus;
            m10 += u * (plus + minus);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

// ---------------------------------------------------------------- GaussianBlur 7x7 sigma 2, 8U
const int kGauss7[7] = {18, 34, 48, 56, 48, 34, 18};  // Q8, sums to 256

inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

void blur7(const uint8_t* src, int w, int h, uint8_t* dst) {
    std::vector<int> tmp((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int i = 0; i < 7; ++i) s += kGauss7[i] * src[(size_t)y * w + reflect101(x + i - 3, w)];
            tmp[(size_t)y * w + x] = s;
        }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int j = 0; j < 7; ++j) s += kGauss7[j] * tmp[(size_t)reflect101(y + j - 3, h) * w + x];
            dst[(size_t)y * w + x] = (uint8_t)((s + 32768) >> 16);
        }
}

// ---------------------------------------------------------------- computeOrbDescriptor (:108-147)
void orb_descriptor(const uint8_t* blur, int w, int cx, int cy, float angleDeg, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    const float ang = angleDeg * factorPI;
    const float a = glibc_cosf(ang), b = glibc_sinf(ang);
    const uint8_t* c = blur + (size_t)cy * w + cx;
    auto value = [&](int idx) {
        const float px = (float)kPattern[2 * idx], py = (float)kPattern[2 * idx + 1];
        const int r = round_even_f(std::fma(px, b, py * a));
        const int q = round_even_f(std::fma(px, a, -(py * b)));
        return (int)c[r * w + q];
    };
    for (int i = 0; i < 32; ++i) {
        int byte = 0;
        for (int k = 0; k < 8; ++k) {
            const int idx = 16 * i + 2 * k;
            byte |= (value(idx) < value(idx + 1)) << k;
        }
        desc[i] = (uint8_t)byte;
    }
}

thread_local std::vector<Image> g_lastPyr;

}  // namespace

// ================================================================ C ABI
extern "C" {

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
float oracle_cosf(float x) { return glibc_cosf(x); }
float oracle_sinf(float x) { return glibc_sinf(x); }

int oracle_tables(const orbfe_params* p, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                  int32_t* n_per_level, int32_t* umax16) {
    Config C;
    if (!make_config(p, C)) return ORBFE_EINVAL;
    for (int l = 0; l < C.nlevels; ++l) {
        if (scale) scale[l] = C.sf[l];
        if (inv_scale) inv_scale[l] = C.isf[l];
        if (sigma2) sigma2[l] = C.s2[l];
        if (inv_sigma2) inv_sigma2[l] = C.is2[l];
        if (n_per_level) n_per_level[l] = C.nPerLevel[l];
    }
    if (umax16)
        for (int v = 0; v <= kHalfPatch; ++v) umax16[v] = C.umax[v];
    return ORBFE_OK;
}

int oracle_level_sizes(const orbfe_params* p, int32_t w, int32_t h, int32_t* wh) {
    Config C;
    if (!make_config(p, C)) return ORBFE_EINVAL;
    for (int l = 0; l < C.nlevels; ++l) {
        wh[2 * l] = round_even_f((float)w * C.isf[l]);
        wh[2 * l + 1] = round_even_f((float)h * C.isf[l]);
    }
    return ORBFE_OK;
}

int oracle_resize(const uint8_t* src, int32_t sw, int32_t sh, int32_t sstride, uint8_t* dst, int32_t dw, int32_t dh,
                  int32_t simd_lanes) {
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return ORBFE_EINVAL;
    resize_linear(src, sw, sh, sstride, dst, dw, dh, simd_lanes);
    return ORBFE_OK;
}

int oracle_blur7(const uint8_t* src, int32_t w, int32_t h, uint8_t* dst) {
    if (w <= 0 || h <= 0) return ORBFE_EINVAL;
    blur7(src, w, h, dst);
    return ORBFE_OK;
}

int oracle_fast(const uint8_t* img, int32_t stride, int32_t w, int32_t h, int32_t th, int32_t* xys, int32_t cap) {
    std::vector<int> out;
    const int n = fast_roi(img, stride, w, h, th, out);
    if (n > cap) return ORBFE_ECAPACITY;
    std::copy(out.begin(), out.end(), xys);
    return n;
}

int oracle_level_candidates(const orbfe_params* p, const uint8_t* lvl, int32_t w, int32_t h, int32_t* xyr,
                            int32_t cap) {
    Config C;
    if (!make_config(p, C)) return ORBFE_EINVAL;
    Image L;
    L.w = w;
    L.h = h;
    L.px.assign(lvl, lvl + (size_t)w * h);
    std::vector<Cand> keys;
    int minX, maxX, minY, maxY;
    level_candidates(C, L, keys, minX, maxX, minY, maxY);
    if ((int)keys.size() > cap) return ORBFE_ECAPACITY;
    for (size_t k = 0; k < keys.size(); ++k) {
        xyr[3 * k] = (int)keys[k].x;
        xyr[3 * k + 1] = (int)keys[k].y;
        xyr[3 * k + 2] = (int)keys[k].resp;
    }
    return (int)keys.size();
}

int oracle_octree(const int32_t* xyr, int32_t n, int32_t minX, int32_t maxX, int32_t minY, int32_t maxY, int32_t N,
                  int32_t* out, int32_t cap) {
    std::vector<Cand> K(n);
    for (int k = 0; k < n; ++k) K[k] = Cand{(float)xyr[3 * k], (float)xyr[3 * k + 1], (float)xyr[3 * k + 2]};
    std::vector<int> sel = distribute(K, minX, maxX, minY, maxY, N);
    if ((int)sel.size() > cap) return ORBFE_ECAPACITY;
    for (size_t i = 0; i < sel.size(); ++i) {
        out[3 * i] = xyr[3 * sel[i]];
        out[3 * i + 1] = xyr[3 * sel[i] + 1];
        out[3 * i + 2] = xyr[3 * sel[i] + 2];
    }
    return (int)sel.size();
}

// The reference runs DistributeOctTree on every level, with or without cells: nIni = round((float)(maxX -
// minX) / (maxY - minY)) sizes vpIniNodes.resize(nIni) (ORBextractor.cpp:543-550), which throws
// std::length_error when nIni < 0 (a level lower than 32 px but wider) and is undefined when maxY == minY; a
// level with cells and nIni == 0 indexes vpIniNodes out of range (:557).  Such geometries are refused.
bool reference_geometry_ok(const Config& C, int W, int H) {
    for (int l = 0; l < C.nlevels; ++l) {
        const int w = round_even_f((float)W * C.isf[l]), h = round_even_f((float)H * C.isf[l]);
        if (w < 1 || h < 1) return false;  // cv::resize of an empty size asserts
        const int sx = (w - kEdge + 3) - (kEdge - 3), sy = (h - kEdge + 3) - (kEdge - 3);
        if (sy == 0) return false;
        const float q = std::round((float)sx / (float)sy);
        if (!std::isfinite(q) || q < 0.f) return false;
        const int nCols = (int)((float)sx / 30.f), nRows = (int)((float)sy / 30.f);
        if (nCols > 0 && nRows > 0 && (int)q == 0) return false;
    }
    return true;
}

int oracle_octree_ties(const orbfe_params* p, const uint8_t* img, int32_t w, int32_t h, int32_t stride, int32_t* ties) {
    Config C;
    if (!make_config(p, C) || !ties) return ORBFE_EINVAL;
    if (w > 0 && h > 0 && !reference_geometry_ok(C, w, h)) return ORBFE_EINVAL;
    for (int l = 0; l < 5 * C.nlevels; ++l) ties[l] = 0;
    if (w <= 0 || h <= 0) return ORBFE_OK;
    std::vector<Image> pyr;
    build_pyramid(C, img, w, h, stride, pyr);
    for (int l = 0; l < C.nlevels; ++l) {
        std::vector<Cand> keys;
        int minX, maxX, minY, maxY;
        level_candidates(C, pyr[l], keys, minX, maxX, minY, maxY);
        TieStats ts;
        distribute(keys, minX, maxX, minY, maxY, C.nPerLevel[l], &ts);
        ties[5 * l] = ts.straddle;
        ties[5 * l + 1] = ts.tie_runs;
        ties[5 * l + 2] = ts.careful_iters;
        ties[5 * l + 3] = ts.run_len;
        ties[5 * l + 4] = ts.run_divided;
    }
    return ORBFE_OK;
}

int oracle_extract(const orbfe_params* p, const uint8_t* img, int32_t w, int32_t h, int32_t stride,
                   orbfe_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out, uint8_t* pyr_out) {
    Config C;
    if (!make_config(p, C) || !n_out) return ORBFE_EINVAL;
    *n_out = 0;
    if (w <= 0 || h <= 0) return ORBFE_OK;  // _image.empty() -> return (:1045-1046)
    if (!reference_geometry_ok(C, w, h)) return ORBFE_EINVAL;
    std::vector<Image>& pyr = g_lastPyr;
    build_pyramid(C, img, w, h, stride, pyr);
    if (pyr_out) {
        size_t o = 0;
        for (const Image& L : pyr) {
            std::memcpy(pyr_out + o, L.px.data(), L.px.size());
            o += L.px.size();
        }
    }
    // ComputeKeyPointsOctTree (:764-852): per level candidates -> octree -> border/octave/size
    struct Sel { int x, y; float resp; };
    std::vector<std::vector<Sel> > all(C.nlevels);
    for (int l = 0; l < C.nlevels; ++l) {
        std::vector<Cand> keys;
        int minX, maxX, minY, maxY;
        level_candidates(C, pyr[l], keys, minX, maxX, minY, maxY);
        std::vector<int> sel = distribute(keys, minX, maxX, minY, maxY, C.nPerLevel[l]);
        for (int k : sel) all[l].push_back(Sel{(int)keys[k].x + minX, (int)keys[k].y + minY, keys[k].resp});
    }
    int total = 0;
    for (auto& v : all) total += (int)v.size();
    if (total > cap) {
        *n_out = total;
        return ORBFE_ECAPACITY;
    }
    // operator_kd (:1074-1103): per level blur + descriptors, then scale coordinates
    int o = 0;
    std::vector<uint8_t> blurred;
    for (int l = 0; l < C.nlevels; ++l) {
        if (all[l].empty()) continue;
        const Image& L = pyr[l];
        blurred.resize(L.px.size());
        blur7(L.px.data(), L.w, L.h, blurred.data());
        const float size = (float)(int)(kPatchSize * C.sf[l]);
        for (const Sel& s : all[l]) {
            orbfe_keypoint& k = kps[o];
            k.angle = ic_angle(L, s.x, s.y, C.umax);
            orb_descriptor(blurred.data(), L.w, s.x, s.y, k.angle, desc + 32 * (size_t)o);
            k.x = (float)s.x;
            k.y = (float)s.y;
            if (l != 0) {
                k.x *= C.sf[l];
                k.y *= C.sf[l];
            }
            k.size = size;
            k.response = s.resp;
            k.octave = l;
            ++o;
        }
    }
    *n_out = o;
    return ORBFE_OK;
}

}  // extern "C"
