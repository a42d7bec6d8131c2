// Device scratch management shared by the check and expand launchers.
#include <cstdio>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "engine.hpp"

namespace keto {

int num_cus(int device) {
    static int cached[64] = {0};
    if (device >= 0 && device < 64 && cached[device]) return cached[device];
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    if (device >= 0 && device < 64) cached[device] = cus;
    return cus;
}

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Allocate (once) disjoint per-tier regions: [ctrl][epochs t0..t2][vis t0][stack t0]...
// Zero-filled at allocation: every epoch starts at 0, so every visited tag is stale.
void ensure_scratch(Scratch &sc, const Tier t[3]) {
    if (sc.mem) return;
    size_t bytes = 256;
    for (int i = 0; i < 3; i++) bytes += align256((size_t)t[i].lanes * 4);
    for (int i = 0; i < 3; i++) bytes += align256((size_t)t[i].lanes * t[i].vcap * 8ull) + align256((size_t)t[i].lanes * t[i].scap * 16ull);
    KETO_HIP(hipMalloc(&sc.mem, bytes));
    KETO_HIP(hipMemset(sc.mem, 0, bytes));
    // the interpreters run on non-blocking streams, which do not wait for the null stream:
    // the zero fill must be complete before any of them can read an epoch or visited slot
    KETO_HIP(hipDeviceSynchronize());
    sc.bytes = bytes;
    char *p = static_cast<char *>(sc.mem);
    sc.ctrl = reinterpret_cast<uint32_t *>(p);
    p += 256;
    for (int i = 0; i < 3; i++) {
        sc.t[i] = t[i];
        sc.epochs[i] = reinterpret_cast<uint32_t *>(p);
        p += align256((size_t)t[i].lanes * 4);
    }
    for (int i = 0; i < 3; i++) {
        sc.vis[i] = reinterpret_cast<unsigned long long *>(p);
        p += align256((size_t)t[i].lanes * t[i].vcap * 8ull);
        sc.stack[i] = reinterpret_cast<uint4 *>(p);
        p += align256((size_t)t[i].lanes * t[i].scap * 16ull);
    }
}

void ensure_lists(Stream &st, uint64_t n) {
    if (st.list_cap >= n) return;
    if (st.lists) KETO_HIP(hipFree(st.lists));
    st.lists = nullptr;
    st.list_cap = 0;
    // [lists 2n u32][ctrl 64 B][resolved 2n uint4]
    const size_t head = align256(2 * n * sizeof(uint32_t) + 64);
    KETO_HIP(hipMalloc(&st.lists, head + 2 * n * sizeof(uint4)));
    st.order_ctrl = st.lists + 2 * n;
    st.resolved = reinterpret_cast<uint4 *>(reinterpret_cast<char *>(st.lists) + head);
    st.list_cap = n;
}

// ---- snapshot array pool ----------------------------------------------------------------------
// A fresh multi-GB device allocation is cleared by the driver before first use (~10 GB/s), so a
// snapshot patched from a base pays seconds for its new arrays unless they come from memory
// the process already holds.  Released snapshot arrays therefore go back to a per-device pool
// (capped at a third of the device), and a store reserves the blocks its next patch needs when
// it cuts a snapshot -- off the transaction path.
namespace {
struct PoolBlock {
    void *p;
    size_t bytes;
};
struct DevicePool {
    std::mutex mu;
    std::vector<PoolBlock> free;
    size_t held = 0, cap = 0;
};
DevicePool &pool_slot(int device) {
    static DevicePool pools[64];
    return pools[std::clamp(device, 0, 63)];
}
DevicePool &pool(int device) {
    DevicePool &P = pool_slot(device);
    if (!P.cap) {  // (KETO_POOL_CAP_MB: processes that share one device, e.g. test ranks, each hold less)
        size_t fr = 0, total = 0;
        const char *e = getenv("KETO_POOL_CAP_MB");
        P.cap = e ? std::max<size_t>((size_t)strtoull(e, nullptr, 10) << 20, 1)
                  : hipMemGetInfo(&fr, &total) == hipSuccess ? total / 3 : (size_t)32 << 30;
    }
    return P;
}
// a free block holding `bytes` without wasting more than half of it
bool take(DevicePool &P, size_t bytes, void **out, size_t *got) {
    size_t best = SIZE_MAX, at = 0;
    for (size_t i = 0; i < P.free.size(); i++)
        if (P.free[i].bytes >= bytes && P.free[i].bytes <= bytes + bytes / 2 && P.free[i].bytes < best) {
            best = P.free[i].bytes;
            at = i;
        }
    if (best == SIZE_MAX) return false;
    *out = P.free[at].p;
    *got = best;
    P.held -= best;
    P.free.erase(P.free.begin() + (ptrdiff_t)at);
    return true;
}
}  // namespace

void *pool_acquire(int device, size_t bytes, size_t *got) {
    DevicePool &P = pool(device);
    {
        std::lock_guard<std::mutex> g(P.mu);
        void *q = nullptr;
        if (take(P, bytes, &q, got)) return q;
        static const bool verbose = getenv("KETO_PATCH_VERBOSE") != nullptr;
        if (verbose) {  // (where a patch's time goes: a miss is a fresh, driver-cleared allocation)
            fprintf(stderr, "[keto pool] miss: %zu bytes; %zu held in", bytes, P.held);
            for (const PoolBlock &b : P.free) fprintf(stderr, " %zu", b.bytes);
            fprintf(stderr, "\n");
        }
    }
    void *q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) {  // out of memory: hand the pool back and try again
        (void)hipGetLastError();
        pool_trim(device);
        KETO_HIP(hipMalloc(&q, bytes));
    }
    *got = bytes;
    return q;
}

// ---- build scratch cache ----------------------------------------------------------------------
// The builder's temporaries (DevBuf) come and go every build; hipFree of a large block unmaps it
// (~0.3 ms each: 5 ms of a config-5 batch's closure build went to them) and synchronises the
// whole device (so a pipelined partition batch's build would wait for the next batch's closure
// kernels at every small free).  Freed blocks stay in a per-device cache instead (capped:
// KETO_SCRATCH_CAP_MB, default a sixteenth of the device), handed out again best-fit within 2x.
// A returned block may still be read by queued kernels: it carries an event recorded on the
// stream the releasing thread works on (scratch_stream; the null stream by default), and its
// next user waits for that event -- not for the whole device.
namespace {
struct CacheBlock {
    void *p;
    size_t bytes;
    hipEvent_t ev;   // nullptr: nothing to wait for
    hipStream_t st;  // the stream ev was recorded on
};
struct ScratchCache {
    std::mutex mu;
    std::vector<CacheBlock> free;
    std::vector<hipEvent_t> events;  // spare events
    size_t held = 0, cap = 0;
};
thread_local hipStream_t tl_stream = nullptr;
ScratchCache &scache_slot(int device) {
    static ScratchCache caches[64];
    return caches[std::clamp(device, 0, 63)];
}
ScratchCache &scache(int device) {
    ScratchCache &C = scache_slot(device);
    if (!C.cap) {
        size_t fr = 0, total = 0;
        const char *e = getenv("KETO_SCRATCH_CAP_MB");
        C.cap = e ? std::max<size_t>((size_t)strtoull(e, nullptr, 10) << 20, 1)
                  : hipMemGetInfo(&fr, &total) == hipSuccess ? total / 16 : (size_t)8 << 30;
    }
    return C;
}
void scratch_trim(int device) {
    ScratchCache &C = scache(device);
    std::lock_guard<std::mutex> g(C.mu);
    if (C.free.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto &b : C.free) {
        (void)hipFree(b.p);
        if (b.ev) C.events.push_back(b.ev);
    }
    C.free.clear();
    C.held = 0;
}
}  // namespace

hipStream_t scratch_stream(hipStream_t s) {
    const hipStream_t old = tl_stream;
    tl_stream = s;
    return old;
}

void *scratch_get(size_t bytes, size_t *got) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        ScratchCache &C = scache(dev);
        std::unique_lock<std::mutex> g(C.mu);
        size_t best = SIZE_MAX, at = 0;
        for (size_t i = 0; i < C.free.size(); i++)
            if (C.free[i].bytes >= bytes && C.free[i].bytes <= 2 * bytes && C.free[i].bytes < best) {
                best = C.free[i].bytes;
                at = i;
            }
        if (best != SIZE_MAX) {
            const CacheBlock b = C.free[at];
            C.held -= best;
            C.free.erase(C.free.begin() + (ptrdiff_t)at);
            // its last reader's stream got past the release -- waited for under the lock, so a
            // stream being destroyed (scratch_forget_stream takes the lock first) is either still
            // alive here or has already retired this event
            if (b.ev) KETO_HIP(hipEventSynchronize(b.ev));
            if (b.ev) C.events.push_back(b.ev);
            *got = best;
            return b.p;
        }
    }
    void *q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) {  // out of memory: the caches' spare blocks go first
        (void)hipGetLastError();
        pool_trim(dev);
        KETO_HIP(hipMalloc(&q, bytes));
    }
    *got = bytes;
    return q;
}

void scratch_put(void *p, size_t bytes) {
    if (!p) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    ScratchCache &C = scache(dev);
    std::lock_guard<std::mutex> g(C.mu);
    if (C.held + bytes <= C.cap) {
        hipEvent_t ev = nullptr;
        if (!C.events.empty()) {
            ev = C.events.back();
            C.events.pop_back();
        } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
        }
        if (ev && hipEventRecord(ev, tl_stream) == hipSuccess) {
            C.free.push_back(CacheBlock{p, bytes, ev, tl_stream});
            C.held += bytes;
            return;
        }
        if (ev) C.events.push_back(ev);
    }
    (void)hipFree(p);
}

// Before stream s is destroyed: the cached blocks whose event was recorded on s wait for it now
// and drop the event (an event whose stream is gone must not be waited on: the runtime then
// reads the dead stream's state -- seen as "operation not permitted on an event last recorded
// in a capturing stream" in a later build).
void scratch_forget_stream(hipStream_t s) {
    if (!s) return;
    for (int d = 0; d < 64; d++) {
        ScratchCache &C = scache_slot(d);
        if (!C.cap) continue;
        std::lock_guard<std::mutex> g(C.mu);
        for (auto &b : C.free)
            if (b.ev && b.st == s) {
                (void)hipEventSynchronize(b.ev);
                C.events.push_back(b.ev);
                b.ev = nullptr;
            }
    }
}

void pool_trim(int device) {
    scratch_trim(device);
    DevicePool &P = pool(device);
    std::lock_guard<std::mutex> g(P.mu);
    if (P.free.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto &b : P.free) (void)hipFree(b.p);
    P.free.clear();
    P.held = 0;
}

// keto_shutdown: every cached block and spare event of every device this process touched goes
// back to the runtime now, while it is certainly alive -- not left to the HIP runtime's own
// teardown in exit(), which runs after the interpreter (and under rocprofv3 after its tool)
// has begun to unwind.  The caches stay usable: a later call simply allocates again.
void pool_shutdown() {
    int cur = 0;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;  // (restored: the caller's thread stays on its device)
    for (int d = 0; d < 64; d++) {
        DevicePool &P = pool_slot(d);
        ScratchCache &C = scache_slot(d);
        if (!P.cap && !C.cap) continue;  // never used on this device
        if (hipSetDevice(d) != hipSuccess) continue;
        pool_trim(d);
        std::lock_guard<std::mutex> g(C.mu);
        for (hipEvent_t e : C.events) (void)hipEventDestroy(e);
        C.events.clear();
    }
    if (have_cur) (void)hipSetDevice(cur);
}

void pool_release(int device, void *p, size_t bytes) {
    if (!p) return;
    DevicePool &P = pool(device);
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();  // (as hipFree would: no kernel may still read it)
    std::lock_guard<std::mutex> g(P.mu);
    if (bytes >= ((size_t)64 << 20) && P.held + bytes <= P.cap) {
        P.free.push_back(PoolBlock{p, bytes});
        P.held += bytes;
    } else {
        (void)hipFree(p);
    }
}

void pool_reserve(int device, const std::vector<size_t> &sizes) {
    DevicePool &P = pool(device);
    std::vector<size_t> need;
    {
        std::lock_guard<std::mutex> g(P.mu);
        std::vector<bool> used(P.free.size(), false);
        for (size_t want : sizes) {
            if (want < ((size_t)64 << 20)) continue;
            bool ok = false;
            for (size_t i = 0; i < P.free.size() && !ok; i++)
                if (!used[i] && P.free[i].bytes >= want && P.free[i].bytes <= want + want / 2) used[i] = ok = true;
            if (!ok) need.push_back(want);
        }
    }
    for (size_t want : need) {
        void *q = nullptr;
        if (hipMalloc(&q, want) != hipSuccess) {
            (void)hipGetLastError();
            return;  // no room for the spare: the patch allocates when it runs
        }
        KETO_HIP(hipMemset(q, 0, want));  // (first touch now, not in the patch)
        pool_release(device, q, want);
    }
}

}  // namespace keto
