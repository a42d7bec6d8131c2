// Microbenchmark (tool, not product): loaded latency of dependent random 16-byte loads on
// gfx950 as a function of the footprint, the waves per CU, the independent loads per step
// and lane-private vs shared regions -- the access pattern of the Check interpreters.
//
//   chase <footprint_MiB> <waves_per_simd> <loads_per_step 1..8> <steps> [private_bytes_per_lane] [width 1|2|4]
//
// Each lane walks `steps` dependent steps; step k loads 1 or 2 random 16-byte windows whose
// addresses depend on the previous step's data (a hash of it), like the interpreters' load
// slot.  With private_bytes_per_lane > 0 every lane stays inside its own region (the
// per-lane visited tables); otherwise addresses span the whole footprint.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    return x;
}

__global__ __launch_bounds__(256) void chase(const uint4 *buf, unsigned long long n_win, int loads, int steps,
                                             unsigned long long priv_win, unsigned int *out, int width) {
    const unsigned long long gl = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    unsigned long long h = mix(gl + 1);
    unsigned int acc = 0;
    const unsigned long long base = priv_win ? (gl * priv_win) % (n_win - priv_win + 1) : 0;
    const unsigned long long span = (priv_win ? priv_win : n_win) - (width - 1);
    for (int k = 0; k < steps; k++) {
        // `loads` independent random windows per step (1..8), each `width` x 16 B contiguous
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            v[j] = make_uint4(0, 0, 0, 0);
            if (j < loads) {
                const unsigned long long i = base + mix(h + j) % span;
                v[j] = buf[i];
                if (width > 1) { const uint4 u = buf[i + 1]; v[j].x ^= u.y; }
                if (width > 2) { const uint4 u = buf[i + 2], w = buf[i + 3]; v[j].y ^= u.z ^ w.w; }
            }
        }
        unsigned long long x = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) x ^= v[j].x ^ ((unsigned long long)v[j].y << 17);
        h = mix(h ^ x ^ (unsigned long long)k);
        acc += (unsigned)x;
    }
    out[gl] = acc;
}

__global__ void fill(uint4 *buf, unsigned long long n) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        buf[i] = make_uint4((unsigned)i, (unsigned)(i * 3), (unsigned)(i * 7), (unsigned)(i * 11));
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: chase MiB waves_per_simd loads steps [private_bytes]\n");
        return 2;
    }
    const unsigned long long bytes = strtoull(argv[1], 0, 10) << 20;
    const int wps = atoi(argv[2]), loads = atoi(argv[3]), steps = atoi(argv[4]);
    const unsigned long long priv = argc > 5 ? strtoull(argv[5], 0, 10) : 0;
    const int width = argc > 6 ? atoi(argv[6]) : 1;  // 16-B windows per access: 1, 2 or 4 (64 B)
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned long long n_win = bytes / 16;
    uint4 *buf;
    CK(hipMalloc(&buf, bytes));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, buf, n_win);
    const unsigned lanes = (unsigned)cus * 4 * wps * 64;
    unsigned int *out;
    CK(hipMalloc(&out, lanes * 4ull));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(chase, dim3(lanes / 256), dim3(256), 0, 0, buf, n_win, loads, steps, priv / 16, out, width);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double ns_step = best * 1e6 / steps;
    const double lines = (double)lanes * steps * loads;
    printf("footprint %6llu MiB waves/SIMD %d loads %d width %2d B private %6llu B: %8.1f ns/step, %.2f G accesses/s, "
           "%.0f GB/s useful\n",
           bytes >> 20, wps, loads, 16 * width, priv, ns_step, lines / (best * 1e-3) / 1e9,
           lines * 16 * width / (best * 1e-3) / 1e9);
    return 0;
}
