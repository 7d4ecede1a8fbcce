// orbfe_host_util.h — error plumbing and device buffers shared by the host translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <new>
#include <stdexcept>
#include <string>

#include "../../include/orbfe.h"

namespace orbfe {

// message of the last failed call on this thread (orbfe_last_error)
extern thread_local std::string g_err;

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCK(expr)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            throw ::orbfe::Error(ORBFE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

template <class F>
int guarded(F&& f) {
    try {
        f();
        return ORBFE_OK;
    } catch (const Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host allocation failed";
        return ORBFE_ENOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return ORBFE_EINVAL;
    }
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void ensure(size_t count) {
        if (count <= n && p) return;
        release();
        if (count == 0) count = 1;
        hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            throw Error(ORBFE_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        n = count;
    }
};

// Page-locked host buffer (hipHostMalloc): the per-frame results come back with asynchronous copies
// into it and one stream synchronisation.
template <class T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0;
    ~HostBuf() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    void ensure(size_t count) {
        if (count <= n && p) return;
        release();
        if (count == 0) count = 1;
        hipError_t e = hipHostMalloc((void**)&p, count * sizeof(T), hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            throw Error(ORBFE_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        }
        n = count;
    }
};

}  // namespace orbfe
