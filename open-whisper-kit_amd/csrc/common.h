// Shared host/device definitions for the MI355X (gfx950) Whisper engine.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#define OWK_HIP_CHECK(expr)                                                                  \
    do {                                                                                     \
        hipError_t owk_err_ = (expr);                                                        \
        if (owk_err_ != hipSuccess) {                                                        \
            char owk_buf_[512];                                                              \
            snprintf(owk_buf_, sizeof(owk_buf_), "HIP error %s at %s:%d: %s",                 \
                     hipGetErrorString(owk_err_), __FILE__, __LINE__, #expr);                \
            throw std::runtime_error(owk_buf_);                                              \
        }                                                                                    \
    } while (0)

namespace owk {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// host-side IEEE binary16 conversion (round-to-nearest-even), identical to the
// F16C/_cvtss_sh path the reference uses for GGML_CPU_FP32_TO_FP16.
static inline uint16_t f32_to_f16_host(float f) {
    _Float16 h = (_Float16) f;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    return u;
}
static inline float f16_to_f32_host(uint16_t u) {
    _Float16 h;
    __builtin_memcpy(&h, &u, 2);
    return (float) h;
}

// RAII device allocation
struct DevBuf {
    void * ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf & operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (ptr) (void) hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    void alloc(size_t n) {
        if (n <= bytes && ptr) return;
        release();
        if (n == 0) return;
        OWK_HIP_CHECK(hipMalloc(&ptr, n));
        bytes = n;
    }
    template <typename T> T * as() const { return (T *) ptr; }
};

// RAII pinned (page-locked) host allocation: async H2D/D2H copies from it are true DMA
struct PinnedBuf {
    void * ptr = nullptr;
    size_t bytes = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf & operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() { release(); }
    void release() {
        if (ptr) (void) hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    void alloc(size_t n) {
        if (n <= bytes && ptr) return;
        release();
        if (n == 0) return;
        OWK_HIP_CHECK(hipHostMalloc(&ptr, n, hipHostMallocDefault));
        bytes = n;
    }
    template <typename T> T * as() const { return (T *) ptr; }
};

// Kernel-bound timing (the selected-class measurement of owk_prof_select / bench.py): while armed,
// launches go through hipExtLaunchKernel with the events bound to the dispatches themselves, so
// hipEventElapsedTime(start, stop) spans the first bracketed kernel's start to the last one's end --
// the dispatch timestamps rocprofv3 reports, without the marker packets of hipEventRecord
struct KTimer {
    hipEvent_t start = nullptr, stop = nullptr;  // stop == nullptr: disarmed
    int launches = 0;
};
inline KTimer * ktimer() {
    static thread_local KTimer t;
    return &t;
}

} // namespace owk

#define OWK_LAUNCH(K, G, B, SHM, ST, ...)                                                            \
    do {                                                                                             \
        ::owk::KTimer * owk_kt_ = ::owk::ktimer();                                                   \
        if (__builtin_expect(owk_kt_->stop != nullptr, 0)) {                                         \
            hipExtLaunchKernelGGL(K, G, B, SHM, ST, owk_kt_->launches == 0 ? owk_kt_->start : nullptr, \
                                  owk_kt_->stop, 0, __VA_ARGS__);                                    \
            owk_kt_->launches++;                                                                     \
        } else {                                                                                     \
            hipLaunchKernelGGL(K, G, B, SHM, ST, __VA_ARGS__);                                       \
        }                                                                                            \
    } while (0)
