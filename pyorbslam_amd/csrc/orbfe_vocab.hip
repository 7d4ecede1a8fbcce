// orbfe_vocab.hip — bag-of-words vocabulary tree on gfx950: native text loader, device node tables and
// the batched descent kernel behind pyDBoW.TemplatedVocabulary.transform (TemplatedVocabulary.py:108-160).
//
// Layout.  The reference keeps Python Node objects with a child-id list each and, per level of a
// descent, computes a per-byte Python popcount against every child (FORB.distance, FORB.py:30-32).
// Here the children of every node occupy one contiguous run of "slots" (slot order = child order), so a
// level of a descent reads count x 32 descriptor bytes in one coalesced sweep:
//   slot_desc[s]  32 B   descriptor of the child in slot s
//   slot_info[s]  16 B   {child node id, its first slot, its child count, its word id}
//   weight[node]  f64    node weight (TemplatedVocabulary.py:67, a Python float)
// The root's run is passed by value.  Host copies of the parsed tables stay in the object (for
// orbfe_vocab_get_nodes and the CPU tests); the device copy is made on first use.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "orbfe_host_util.h"

using namespace orbfe;

struct orbfe_vocab {
    orbfe_vocab_info info{};
    // per node (id order, entry 0 = root)
    std::vector<int32_t> parent;
    std::vector<uint8_t> leaf_flag;
    std::vector<uint8_t> desc;      // 32 B per node
    std::vector<double> weight;
    std::vector<int32_t> word;
    // per slot
    std::vector<int4> slot_info;
    int32_t root_count = 0;
    // device
    bool uploaded = false;
    DevBuf<uint4> d_slot_desc;
    DevBuf<int4> d_slot_info;
    DevBuf<double> d_weight;
    DevBuf<uint8_t> d_q;
    DevBuf<int32_t> d_word, d_node;
    DevBuf<double> d_w;
    hipStream_t stream = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    float last_ms = 0.f;
    // transform callers share one vocabulary across threads (Frame.compute_BoW on the tracking thread,
    // KeyFrame.compute_bow on the mapping thread: Frame.py:125, KeyFrame.py:119): the scratch buffers,
    // the stream and the events above are guarded by this mutex
    std::mutex mu;
    ~orbfe_vocab() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace orbfe {

constexpr int kVocabPerBlock = 8;  // descriptors per 256-thread block: 32 lanes each

// One descent per 32-lane group.  Per level, lane j takes child j (j, j+32, ... when a node has more
// than 32 children), XORs its 32 descriptor bytes with the query and counts bits (v_bcnt accumulate);
// the group minimum of key = dist << 16 | child position is the reference's first strict minimum
// (TemplatedVocabulary.py:143-150).  The winner's slot_info was loaded by its own lane together with
// the descriptor, so the next level needs no dependent table read: one memory round trip per level.
__global__ __launch_bounds__(256) void k_vocab_descend(const uint8_t* __restrict__ q, int64_t n, int root_count,
                                                       const uint4* __restrict__ slot_desc,
                                                       const int4* __restrict__ slot_info,
                                                       const double* __restrict__ weight, int nid_level,
                                                       int32_t* __restrict__ out_word, int32_t* __restrict__ out_node,
                                                       double* __restrict__ out_w) {
    const int lane = threadIdx.x & 31;
    const int64_t i = (int64_t)blockIdx.x * kVocabPerBlock + (threadIdx.x >> 5);
    if (i >= n) return;  // the whole 32-lane group leaves together
    const uint4* qp = reinterpret_cast<const uint4*>(q + i * 32);
    const uint4 qa = qp[0], qb = qp[1];
    int node = 0, start = 0, count = root_count, word = 0, nid = -1;
    for (int level = 1; count > 0; ++level) {
        unsigned best = 0xFFFFFFFFu;
        int4 mine = make_int4(0, 0, 0, 0);
        for (int c0 = 0; c0 < count; c0 += 32) {
            const int j = c0 + lane;
            if (j < count) {
                const uint4 a = slot_desc[2 * (start + j)];
                const uint4 b = slot_desc[2 * (start + j) + 1];
                const int4 inf = slot_info[start + j];
                unsigned d = __popc(a.x ^ qa.x) + __popc(a.y ^ qa.y) + __popc(a.z ^ qa.z) + __popc(a.w ^ qa.w) +
                             __popc(b.x ^ qb.x) + __popc(b.y ^ qb.y) + __popc(b.z ^ qb.z) + __popc(b.w ^ qb.w);
                const unsigned key = (d << 16) | (unsigned)j;
                if (key < best) {
                    best = key;
                    mine = inf;
                }
            }
        }
#pragma unroll
        for (int o = 16; o; o >>= 1) best = min(best, (unsigned)__shfl_xor((int)best, o, 32));
        const int wl = (int)(best & 31u);
        node = __shfl(mine.x, wl, 32);
        start = __shfl(mine.y, wl, 32);
        count = __shfl(mine.z, wl, 32);
        word = __shfl(mine.w, wl, 32);
        if (level == nid_level) nid = node;
    }
    if (lane == 0) {
        out_word[i] = word;
        out_node[i] = nid;
        out_w[i] = weight[node];
    }
}

}  // namespace orbfe

namespace {

// Build children runs, word ids, depth from the per-node arrays (validated).
void finish(orbfe_vocab& v) {
    const int64_t n = (int64_t)v.parent.size();
    std::vector<int32_t> nch(n, 0);
    for (int64_t i = 1; i < n; ++i) nch[v.parent[i]]++;
    std::vector<int32_t> first(n, 0);
    int64_t s = 0;
    for (int64_t i = 0; i < n; ++i) {
        first[i] = (int32_t)s;
        s += nch[i];
    }
    v.word.assign(n, 0);
    int64_t nw = 0;
    for (int64_t i = 1; i < n; ++i)
        if (v.leaf_flag[i]) v.word[i] = (int32_t)nw++;
    std::vector<int32_t> fill(n, 0), depth(n, 0);
    v.slot_info.assign(std::max<int64_t>(n - 1, 0), make_int4(0, 0, 0, 0));
    int maxd = 0;
    for (int64_t i = 1; i < n; ++i) {
        const int32_t p = v.parent[i];
        v.slot_info[first[p] + fill[p]++] = make_int4((int)i, first[i], nch[i], v.word[i]);
        depth[i] = depth[p] + 1;
        maxd = std::max(maxd, depth[i]);
    }
    v.root_count = n > 0 ? nch[0] : 0;
    v.info.n_nodes = n;
    v.info.n_words = nw;
    v.info.depth = maxd;
    v.info.max_children = n > 0 ? *std::max_element(nch.begin(), nch.end()) : 0;
    if (v.info.max_children > 65535) throw Error(ORBFE_EINVAL, "more than 65535 children under one node");
}

void upload(orbfe_vocab& v) {
    if (v.uploaded) return;
    if (!v.stream) HIPCK(hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking));
    for (hipEvent_t& e : v.ev)
        if (!e) HIPCK(hipEventCreate(&e));
    const size_t ns = v.slot_info.size();
    std::vector<uint8_t> sd(std::max<size_t>(ns, 1) * 32, 0);
    for (size_t s = 0; s < ns; ++s) std::memcpy(&sd[s * 32], &v.desc[(size_t)v.slot_info[s].x * 32], 32);
    v.d_slot_desc.ensure(std::max<size_t>(ns, 1) * 2);
    v.d_slot_info.ensure(std::max<size_t>(ns, 1));
    v.d_weight.ensure(v.weight.size());
    HIPCK(hipMemcpy(v.d_slot_desc.p, sd.data(), sd.size(), hipMemcpyHostToDevice));
    if (ns) HIPCK(hipMemcpy(v.d_slot_info.p, v.slot_info.data(), ns * sizeof(int4), hipMemcpyHostToDevice));
    HIPCK(hipMemcpy(v.d_weight.p, v.weight.data(), v.weight.size() * sizeof(double), hipMemcpyHostToDevice));
    v.uploaded = true;
}

void launch_descend(orbfe_vocab& v, const uint8_t* d_q, int64_t n, int nid_level, int32_t* d_word, int32_t* d_node,
                    double* d_w, hipStream_t s) {
    if (n <= 0) return;
    const int64_t blocks = (n + kVocabPerBlock - 1) / kVocabPerBlock;
    if (blocks > 0x7FFFFFFF) throw Error(ORBFE_EINVAL, "too many descriptors for one launch");
    hipLaunchKernelGGL(k_vocab_descend, dim3((unsigned)blocks), dim3(256), 0, s, d_q, n, v.root_count,
                       v.d_slot_desc.p, v.d_slot_info.p, v.d_weight.p, nid_level, d_word, d_node, d_w);
    HIPCK(hipGetLastError());
}

// ---- text loader (TemplatedVocabulary.load_from_text_file, TemplatedVocabulary.py:43-81) ----------

// Python int(token): optional sign, decimal digits only.
bool parse_int(const char* b, const char* e, long long& out) {
    if (b == e) return false;
    const char* p = b;
    bool neg = false;
    if (*p == '+' || *p == '-') neg = *p++ == '-';
    if (p == e) return false;
    long long v = 0;
    for (; p < e; ++p) {
        if (*p < '0' || *p > '9') return false;
        v = v * 10 + (*p - '0');
        if (v > (1LL << 40)) return false;
    }
    out = neg ? -v : v;
    return true;
}

// Python float(token) via strtod on a NUL-terminated copy (tokens are short).
bool parse_float(const char* b, const char* e, double& out) {
    char buf[64];
    const size_t len = (size_t)(e - b);
    if (len == 0 || len >= sizeof(buf)) return false;
    std::memcpy(buf, b, len);
    buf[len] = 0;
    char* end = nullptr;
    errno = 0;
    out = std::strtod(buf, &end);
    return end == buf + len;
}

struct Tokens {
    const char* b[40];
    const char* e[40];
    int n = 0;
};

// str.strip().split() of one line, at most 40 tokens (more -> n = 41 marks "too many")
void split(const char* p, const char* end, Tokens& t) {
    t.n = 0;
    while (p < end) {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
        if (p >= end) break;
        const char* s = p;
        while (p < end && !(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
        if (t.n == 40) {
            t.n = 41;
            return;
        }
        t.b[t.n] = s;
        t.e[t.n] = p;
        ++t.n;
    }
}

std::unique_ptr<orbfe_vocab> load_text(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) throw Error(ORBFE_EINVAL, std::string("cannot open vocabulary file: ") + path);
    std::string text;
    {
        char buf[1 << 16];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, r);
        std::fclose(f);
    }
    const char* p = text.data();
    const char* end = p + text.size();
    auto next_line = [&](const char*& b, const char*& e) -> bool {
        if (p >= end) return false;
        b = p;
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        e = nl ? nl : end;
        p = nl ? nl + 1 : end;
        return true;
    };
    auto v = std::make_unique<orbfe_vocab>();
    const char *lb, *le;
    Tokens t;
    if (!next_line(lb, le)) throw Error(ORBFE_EFORMAT, "empty vocabulary file");
    split(lb, le, t);
    long long hv[4];
    if (t.n < 4) throw Error(ORBFE_EFORMAT, "vocabulary header needs 4 integers");
    for (int k = 0; k < 4; ++k)
        if (!parse_int(t.b[k], t.e[k], hv[k])) throw Error(ORBFE_EFORMAT, "vocabulary header is not integer");
    v->info.k = (int32_t)hv[0];
    v->info.L = (int32_t)hv[1];
    v->info.scoring = (int32_t)hv[2];
    v->info.weighting = (int32_t)hv[3];
    if (hv[0] < 0 || hv[0] > 20 || hv[1] < 1 || hv[1] > 10 || hv[2] < 0 || hv[2] > 5 || hv[3] < 0 || hv[3] > 3)
        throw Error(ORBFE_EREJECT, "Vocabulary loading failure: Invalid parameters in file!");
    v->parent.push_back(0);
    v->leaf_flag.push_back(0);
    v->desc.resize(32, 0);
    v->weight.push_back(0.0);
    int64_t line_no = 1;
    while (next_line(lb, le)) {
        ++line_no;
        split(lb, le, t);
        if (t.n != 35)
            throw Error(ORBFE_EFORMAT, "vocabulary line " + std::to_string(line_no) + ": expected 35 fields");
        long long par, leaf;
        if (!parse_int(t.b[0], t.e[0], par) || !parse_int(t.b[1], t.e[1], leaf))
            throw Error(ORBFE_EFORMAT, "vocabulary line " + std::to_string(line_no) + ": bad parent / leaf flag");
        const int64_t id = (int64_t)v->parent.size();
        if (par < 0 || par >= id)
            throw Error(ORBFE_EFORMAT, "vocabulary line " + std::to_string(line_no) + ": parent is not an earlier node");
        uint8_t d[32];
        for (int k = 0; k < 32; ++k) {
            double x;
            if (!parse_float(t.b[2 + k], t.e[2 + k], x) || !(x > -1.0 && x < 256.0))
                throw Error(ORBFE_EFORMAT, "vocabulary line " + std::to_string(line_no) + ": descriptor byte");
            d[k] = (uint8_t)(int)x;  // numpy astype(int): truncation
        }
        double w;
        if (!parse_float(t.b[34], t.e[34], w))
            throw Error(ORBFE_EFORMAT, "vocabulary line " + std::to_string(line_no) + ": weight");
        v->parent.push_back((int32_t)par);
        v->leaf_flag.push_back(leaf > 0 ? 1 : 0);
        v->desc.insert(v->desc.end(), d, d + 32);
        v->weight.push_back(w);
    }
    finish(*v);
    return v;
}

}  // namespace

extern "C" {

int orbfe_vocab_load_text(const char* path, orbfe_vocab_handle* out) {
    return guarded([&] {
        if (!path || !out) throw Error(ORBFE_EINVAL, "null argument");
        *out = load_text(path).release();
    });
}

int orbfe_vocab_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int64_t n_nodes,
                       const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc32, const double* weight,
                       orbfe_vocab_handle* out) {
    return guarded([&] {
        if (!out || n_nodes < 1 || (n_nodes > 1 && (!parent || !is_leaf || !desc32 || !weight)))
            throw Error(ORBFE_EINVAL, "bad argument");
        auto v = std::make_unique<orbfe_vocab>();
        v->info.k = k;
        v->info.L = L;
        v->info.scoring = scoring;
        v->info.weighting = weighting;
        v->parent.assign(n_nodes, 0);
        v->leaf_flag.assign(n_nodes, 0);
        v->desc.assign((size_t)n_nodes * 32, 0);
        v->weight.assign(n_nodes, 0.0);
        for (int64_t i = 1; i < n_nodes; ++i) {
            if (parent[i] < 0 || parent[i] >= i) throw Error(ORBFE_EINVAL, "parent must be an earlier node");
            v->parent[i] = parent[i];
            v->leaf_flag[i] = is_leaf[i] ? 1 : 0;
            std::memcpy(&v->desc[(size_t)i * 32], desc32 + (size_t)i * 32, 32);
            v->weight[i] = weight[i];
        }
        finish(*v);
        *out = v.release();
    });
}

int orbfe_vocab_destroy(orbfe_vocab_handle v) {
    return guarded([&] { delete v; });
}

int orbfe_vocab_get_info(orbfe_vocab_handle v, orbfe_vocab_info* info) {
    return guarded([&] {
        if (!v || !info) throw Error(ORBFE_EINVAL, "null argument");
        *info = v->info;
    });
}

int orbfe_vocab_get_nodes(orbfe_vocab_handle v, int32_t* parent, uint8_t* is_leaf, uint8_t* desc32, double* weight,
                          int32_t* word_id) {
    return guarded([&] {
        if (!v) throw Error(ORBFE_EINVAL, "null argument");
        const size_t n = v->parent.size();
        if (parent) std::memcpy(parent, v->parent.data(), n * sizeof(int32_t));
        if (is_leaf) std::memcpy(is_leaf, v->leaf_flag.data(), n);
        if (desc32) std::memcpy(desc32, v->desc.data(), n * 32);
        if (weight) std::memcpy(weight, v->weight.data(), n * sizeof(double));
        if (word_id) std::memcpy(word_id, v->word.data(), n * sizeof(int32_t));
    });
}

int orbfe_vocab_transform(orbfe_vocab_handle v, const uint8_t* desc32, int64_t n, int32_t nid_level, int32_t* word_id,
                          int32_t* node_id, double* weight) {
    return guarded([&] {
        if (!v || n < 0 || (n > 0 && (!desc32 || !word_id || !node_id || !weight)))
            throw Error(ORBFE_EINVAL, "bad argument");
        if (n == 0) return;
        std::lock_guard<std::mutex> lk(v->mu);
        upload(*v);
        v->d_q.ensure((size_t)n * 32);
        v->d_word.ensure(n);
        v->d_node.ensure(n);
        v->d_w.ensure(n);
        HIPCK(hipMemcpyAsync(v->d_q.p, desc32, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
        HIPCK(hipEventRecord(v->ev[0], v->stream));
        launch_descend(*v, v->d_q.p, n, nid_level, v->d_word.p, v->d_node.p, v->d_w.p, v->stream);
        HIPCK(hipEventRecord(v->ev[1], v->stream));
        HIPCK(hipMemcpyAsync(word_id, v->d_word.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
        HIPCK(hipMemcpyAsync(node_id, v->d_node.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
        HIPCK(hipMemcpyAsync(weight, v->d_w.p, n * sizeof(double), hipMemcpyDeviceToHost, v->stream));
        HIPCK(hipStreamSynchronize(v->stream));
        HIPCK(hipEventElapsedTime(&v->last_ms, v->ev[0], v->ev[1]));
    });
}

int orbfe_vocab_transform_device(orbfe_vocab_handle v, const uint8_t* d_desc32, int64_t n, int32_t nid_level,
                                 int32_t* d_word_id, int32_t* d_node_id, double* d_weight, void* hip_stream) {
    return guarded([&] {
        if (!v || n < 0 || (n > 0 && (!d_desc32 || !d_word_id || !d_node_id || !d_weight)))
            throw Error(ORBFE_EINVAL, "bad argument");
        if (reinterpret_cast<uintptr_t>(d_desc32) & 15) throw Error(ORBFE_EINVAL, "descriptors must be 16-byte aligned");
        std::lock_guard<std::mutex> lk(v->mu);
        upload(*v);
        launch_descend(*v, d_desc32, n, nid_level, d_word_id, d_node_id, d_weight,
                       static_cast<hipStream_t>(hip_stream));
    });
}

int orbfe_vocab_last_ms(orbfe_vocab_handle v, float* ms) {
    return guarded([&] {
        if (!v || !ms) throw Error(ORBFE_EINVAL, "null argument");
        std::lock_guard<std::mutex> lk(v->mu);
        *ms = v->last_ms;
    });
}

}  // extern "C"
