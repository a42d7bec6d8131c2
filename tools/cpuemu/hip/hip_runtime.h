// TEST/DEBUG TOOL ONLY -- not part of the product.
// A minimal host-side stand-in for the HIP runtime so the gfx950 kernel SOURCES in
// djy-keto_amd/csrc can be executed on the CPU, one lane at a time (a wavefront of one
// lane, blockDim 1), to debug interpreter logic against the oracle without a GPU.
// The resulting library (tools/cpuemu/libketo_emu.so) is loaded only when a test sets
// KETO_MI355X_ALLOW_OVERRIDE=tools plus KETO_MI355X_LIB_OVERRIDE; the product never does.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__

struct uint4 {
    uint32_t x, y, z, w;
};
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
struct uint2 {
    uint32_t x, y;
};
inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }
struct dim3 {
    uint32_t x, y, z;
    dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};
struct EmuIdx {
    uint32_t x = 0, y = 0, z = 0;
};
inline thread_local EmuIdx threadIdx, blockIdx, blockDim, gridDim;


typedef int hipError_t;
typedef void *hipStream_t;
typedef void *hipEvent_t;
enum { hipSuccess = 0 };
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice };
enum { hipStreamNonBlocking = 1 };
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount };

inline const char *hipGetErrorString(hipError_t) { return "emu error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipDeviceSynchronize() { return hipSuccess; }
inline hipError_t hipGetDeviceCount(int *n) { *n = 1; return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t, int) { *v = 2; return hipSuccess; }
inline hipError_t hipMalloc(void **p, size_t n) { *p = std::calloc(1, n + 64); return *p ? hipSuccess : 1; }
template <class T>
inline hipError_t hipMalloc(T **p, size_t n) { return hipMalloc(reinterpret_cast<void **>(p), n); }
inline hipError_t hipFree(void *p) { std::free(p); return hipSuccess; }
inline hipError_t hipHostMalloc(void **p, size_t n, unsigned) { return hipMalloc(p, n); }
inline hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
inline hipError_t hipMemGetInfo(size_t *f, size_t *t) { *f = *t = (size_t)64 << 30; return hipSuccess; }
inline hipError_t hipHostFree(void *p) { std::free(p); return hipSuccess; }
// (every emulated allocation is host memory the "device" reaches: pinned-buffer paths run as on the GPU)
enum hipMemoryType { hipMemoryTypeUnregistered = 0, hipMemoryTypeHost = 1, hipMemoryTypeDevice = 2 };
struct hipPointerAttribute_t {
    hipMemoryType type;
    int device;
    void *devicePointer, *hostPointer;
};
inline hipError_t hipPointerGetAttributes(hipPointerAttribute_t *a, const void *p) {
    *a = hipPointerAttribute_t{hipMemoryTypeHost, 0, const_cast<void *>(p), const_cast<void *>(p)};
    return hipSuccess;
}
inline hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyToSymbol(void *sym, const void *s, size_t n, size_t off = 0, hipMemcpyKind = hipMemcpyHostToDevice) { std::memcpy(static_cast<char *>(sym) + off, s, n); return hipSuccess; }
#define HIP_SYMBOL(x) (&(x))
inline hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind, hipStream_t) { std::memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemset(void *d, int v, size_t n) { std::memset(d, v, n); return hipSuccess; }
inline hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t) { std::memset(d, v, n); return hipSuccess; }
// Streams are objects that remember being destroyed (never freed: an event recorded on one may
// outlive it), and waiting on an event whose stream is gone fails -- as the runtime refuses it
// ("operation not permitted on an event last recorded in a capturing stream"), so the library's
// scratch-cache discipline (scratch_forget_stream) is checked on the CPU.
struct EmuStream {
    bool alive = true;
};
struct EmuEvent {
    double t = 0;
    EmuStream *st = nullptr;
};
inline hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = new EmuStream(); return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t s) {
    if (s) static_cast<EmuStream *>(s)->alive = false;
    return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t *e) { *e = new EmuEvent(); return hipSuccess; }
#define hipEventDisableTiming 2u
inline hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { return hipEventCreate(e); }
inline hipError_t hipEventDestroy(hipEvent_t e) { delete static_cast<EmuEvent *>(e); return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    auto *v = static_cast<EmuEvent *>(e);
    v->t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    v->st = static_cast<EmuStream *>(s);
    return hipSuccess;
}
inline hipError_t emu_event_live(hipEvent_t e) {
    const auto *v = static_cast<const EmuEvent *>(e);
    return (v && v->st && !v->st->alive) ? 1 : hipSuccess;
}
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t e, unsigned) { return emu_event_live(e); }
inline hipError_t hipEventSynchronize(hipEvent_t e) { return emu_event_live(e); }
inline hipError_t hipEventQuery(hipEvent_t e) { return emu_event_live(e); }  // (the emulation runs every launch at once)
inline hipError_t hipEventElapsedTime(float *ms, hipEvent_t a, hipEvent_t b) {
    *ms = float(static_cast<EmuEvent *>(b)->t - static_cast<EmuEvent *>(a)->t);
    return hipSuccess;
}
template <class K>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int *n, K, int, size_t) { *n = 2; return hipSuccess; }

// one lane per wavefront
inline uint32_t __lane_id() { return 0; }
inline unsigned long long __ballot(int p) { return p ? 1ull : 0ull; }
template <class T> inline T __shfl(T v, int) { return v; }
template <class T> inline T __shfl_down(T, int) { return T(0); }
template <class T> inline T __shfl_up(T, int) { return T(0); }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
inline int __clzll(long long v) { return v ? __builtin_clzll((unsigned long long)v) : 64; }
inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline void __syncthreads() {}
inline uint32_t atomicAdd(uint32_t *p, uint32_t v) { uint32_t o = *p; *p += v; return o; }
inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) { auto o = *p; *p += v; return o; }
inline unsigned long long atomicOr(unsigned long long *p, unsigned long long v) { auto o = *p; *p |= v; return o; }
inline uint32_t atomicOr(uint32_t *p, uint32_t v) { uint32_t o = *p; *p |= v; return o; }
inline unsigned long long atomicAnd(unsigned long long *p, unsigned long long v) { auto o = *p; *p &= v; return o; }
inline unsigned long long atomicMin(unsigned long long *p, unsigned long long v) { auto o = *p; *p = std::min(o, v); return o; }
inline unsigned long long atomicMax(unsigned long long *p, unsigned long long v) { auto o = *p; *p = std::max(o, v); return o; }
inline uint32_t atomicCAS(uint32_t *p, uint32_t c, uint32_t v) {
    uint32_t o = *p;
    if (o == c) *p = v;
    return o;
}
constexpr int warpSize = 1;
#define __builtin_amdgcn_readfirstlane(x) (x)
#define __builtin_amdgcn_readlane(x, l) (x)
#define __builtin_amdgcn_fence(...) ((void)0)
#define __builtin_amdgcn_s_memtime() 0ull
#define __builtin_amdgcn_wave_barrier() ((void)0)
inline unsigned long long atomicCAS(unsigned long long *p, unsigned long long c, unsigned long long v) {
    auto o = *p;
    if (o == c) *p = v;
    return o;
}

// every lane runs to completion in turn: a persistent lane drains the work queue alone
#define hipLaunchKernelGGL(kernel, grid, block, shmem, stream, ...)                          \
    do {                                                                                      \
        const uint32_t emu_n = dim3(grid).x * dim3(block).x;                                  \
        for (uint32_t emu_g = 0; emu_g < emu_n; emu_g++) {                                    \
            blockIdx.x = emu_g;                                                               \
            threadIdx.x = 0;                                                                  \
            blockDim.x = 1;                                                                   \
            gridDim.x = emu_n;                                                                \
            kernel(__VA_ARGS__);                                                              \
        }                                                                                     \
    } while (0)
