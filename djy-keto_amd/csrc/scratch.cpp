// Device scratch management shared by the check and expand launchers.
#include <hip/hip_runtime.h>

#include <algorithm>

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


}  // namespace keto
