// Stream-ordered device primitives of the partition path (csrc/partition.hip): a stable LSD radix
// sort of (key, value) pairs and sorted-run compaction, hand-written for gfx950 (64-wide waves,
// LDS-staged tiles).  Scans are build.hip's chunked scan (build::scan_excl).
//
// Radix sort, one 8-bit digit per pass (stable, so passes compose from the lowest digit up):
//   k_radix_hist     each block histograms one tile of RTILE keys into LDS bins, written
//                    digit-major: hist[d * tiles + tile];
//   build::scan_excl the digit-major histogram -> every (digit, tile)'s first output position;
//   k_radix_scatter  each block ranks its tile stably in LDS -- per round of 256 keys, a wave's
//                    equal digits are found with 8 ballots and counted with popcounts, the waves
//                    of the round are combined through per-digit counters -- so the tile sits in
//                    LDS sorted by digit, and is then written out run by run: consecutive lanes
//                    store consecutive addresses of one digit's output range (coalesced), not
//                    one scattered word per lane.
// Keys must fit `bits` (the caller's key width): only those digits are sorted.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace prim {
namespace {

using build::DevBuf;
constexpr uint32_t RBLK = 256;              // threads per block = digit bins (one counter per thread)
constexpr uint32_t RBINS = 256;
constexpr uint32_t RITEMS = 16;             // rounds of RBLK keys per tile
constexpr uint32_t RTILE = RBLK * RITEMS;   // 4096 keys per tile
constexpr uint32_t RWAVES = RBLK / 64;

template <class K>
__device__ __forceinline__ uint32_t digit_of(K k, uint32_t shift) {
    return (uint32_t)(k >> shift) & (RBINS - 1u);
}

template <class K>
__global__ __launch_bounds__(RBLK) void k_radix_hist(const K *keys, uint64_t n, uint32_t shift, uint32_t *hist,
                                                     uint32_t tiles) {
    __shared__ uint32_t h[RBINS];
    const uint32_t t = threadIdx.x;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        h[t] = 0;
        __syncthreads();
        const uint64_t base = (uint64_t)tile * RTILE;
        for (uint32_t k = 0; k < RITEMS; k++) {
            const uint64_t i = base + (uint64_t)k * RBLK + t;
            if (i < n) atomicAdd(&h[digit_of(keys[i], shift)], 1u);
        }
        __syncthreads();
        hist[(uint64_t)t * tiles + tile] = h[t];
        __syncthreads();
    }
}

template <class K, class V>
__global__ __launch_bounds__(RBLK) void k_radix_scatter(const K *keys, const V *vals, uint64_t n, uint32_t shift,
                                                        const uint32_t *offs, uint32_t tiles, K *okeys, V *ovals) {
    __shared__ K sk[RTILE];
    __shared__ V sv[RTILE];
    __shared__ uint32_t run[RBINS], loc[RBINS], glob[RBINS], wc[RWAVES][RBINS], wsum[RWAVES + 1];
    const uint32_t t = threadIdx.x, lane = __lane_id(), w = t >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const uint64_t base = (uint64_t)tile * RTILE;
        const uint32_t tn = (uint32_t)min<uint64_t>(RTILE, n - base);
        K kk[RITEMS];
        V vv[RITEMS];
        run[t] = 0;
        __syncthreads();
        for (uint32_t k = 0; k < RITEMS; k++) {
            const uint32_t j = k * RBLK + t;
            if (j < tn) {
                kk[k] = keys[base + j];
                vv[k] = vals[base + j];
                atomicAdd(&run[digit_of(kk[k], shift)], 1u);
            }
        }
        __syncthreads();
        // local digit starts: exclusive scan of the tile's counts (one bin per thread)
        {
            const uint32_t c = run[t];
            uint32_t x = c;
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            if (lane == 63) wsum[w] = x;
            __syncthreads();
            if (t == 0) {
                uint32_t s = 0;
                for (uint32_t i = 0; i < RWAVES; i++) {
                    const uint32_t y = wsum[i];
                    wsum[i] = s;
                    s += y;
                }
            }
            __syncthreads();
            loc[t] = wsum[w] + x - c;
            glob[t] = offs[(uint64_t)t * tiles + tile];
            run[t] = 0;  // keys of each digit placed so far
        }
        __syncthreads();
        // stable ranks, round by round (element order within a tile: round, wave, lane)
        for (uint32_t k = 0; k < RITEMS; k++) {
            for (uint32_t i = t; i < RWAVES * RBINS; i += RBLK) (&wc[0][0])[i] = 0;
            const uint32_t j = k * RBLK + t;
            const bool valid = j < tn;
            const uint32_t d = valid ? digit_of(kk[k], shift) : 0u;
            unsigned long long peer = __ballot(valid);
            for (uint32_t b = 0; b < 8; b++) {
                const unsigned long long bb = __ballot(valid && ((d >> b) & 1u));
                peer &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t wrank = (uint32_t)__popcll(peer & lt);
            __syncthreads();
            if (valid && wrank == 0) wc[w][d] = (uint32_t)__popcll(peer);
            __syncthreads();
            {   // digit t: the waves' counts -> their starts, the running count moves on
                uint32_t s = run[t];
                for (uint32_t i = 0; i < RWAVES; i++) {
                    const uint32_t y = wc[i][t];
                    wc[i][t] = s;
                    s += y;
                }
                run[t] = s;
            }
            __syncthreads();
            if (valid) {
                const uint32_t p = loc[d] + wc[w][d] + wrank;
                sk[p] = kk[k];
                sv[p] = vv[k];
            }
            __syncthreads();  // (the next round clears wc)
        }
        __syncthreads();
        // the tile in digit order, written digit run by digit run
        for (uint32_t j = t; j < tn; j += RBLK) {
            const K x = sk[j];
            const uint32_t d = digit_of(x, shift);
            const uint64_t o = (uint64_t)glob[d] + (j - loc[d]);
            okeys[o] = x;
            ovals[o] = sv[j];
        }
        __syncthreads();
    }
}

// run flags of a sorted array: flag[i] = a[i] != a[i-1]; flag[n] = 0 (scanned into positions)
template <class K>
__global__ __launch_bounds__(RBLK) void k_run_flags(const K *a, uint64_t n, uint32_t *flag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x)
        flag[i] = i < n && (i == 0 || a[i] != a[i - 1]) ? 1u : 0u;
}
template <class K>
__global__ __launch_bounds__(RBLK) void k_run_compact(const K *a, uint64_t n, const uint32_t *pos, K *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (i == 0 || a[i] != a[i - 1]) out[pos[i]] = a[i];
}
__global__ __launch_bounds__(RBLK) void k_sum_u32(const uint32_t *v, uint64_t n, unsigned long long *out) {
    __shared__ unsigned long long s[RWAVES];
    unsigned long long acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) acc += v[i];
    for (uint32_t off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
    if (__lane_id() == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (uint32_t i = 0; i < RWAVES; i++) tot += s[i];
        if (tot) atomicAdd(out, tot);
    }
}

inline dim3 grid_n(uint64_t n, uint32_t cap = 1u << 16) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + RBLK - 1) / RBLK, cap)));
}

template <class K, class V>
bool sort_pairs_impl(K *k0, V *v0, K *k1, V *v1, uint64_t n, uint32_t bits, hipStream_t s) {
    if (n <= 1 || bits == 0) return false;
    if (n >= (1ull << 32)) throw Error(KETO_E_LIMIT, "radix sort of 2^32 or more keys");
    const uint32_t tiles = (uint32_t)((n + RTILE - 1) / RTILE);
    if ((uint64_t)tiles * RBINS >= (1ull << 32)) throw Error(KETO_E_LIMIT, "radix sort histogram too large");
    DevBuf hist(((uint64_t)tiles * RBINS + 1) * 4);
    int dev = 0;
    KETO_HIP(hipGetDevice(&dev));
    const dim3 G(std::min<uint32_t>(tiles, (uint32_t)std::max(1, num_cus(dev)) * 8u));
    bool flip = false;
    for (uint32_t shift = 0; shift < bits; shift += 8) {
        const K *ki = flip ? k1 : k0;
        const V *vi = flip ? v1 : v0;
        K *ko = flip ? k0 : k1;
        V *vo = flip ? v0 : v1;
        hipLaunchKernelGGL(k_radix_hist<K>, G, dim3(RBLK), 0, s, ki, n, shift, hist.u32(), tiles);
        KETO_HIP(hipGetLastError());
        build::scan_excl(hist.u32(), (uint64_t)tiles * RBINS, s);
        hipLaunchKernelGGL((k_radix_scatter<K, V>), G, dim3(RBLK), 0, s, ki, vi, n, shift, hist.u32(), tiles, ko, vo);
        KETO_HIP(hipGetLastError());
        flip = !flip;
    }
    return flip;
}

}  // namespace

bool sort_pairs(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t bits, hipStream_t s) {
    return sort_pairs_impl(k0, v0, k1, v1, n, bits, s);
}
bool sort_pairs(uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, uint32_t bits, hipStream_t s) {
    return sort_pairs_impl(k0, v0, k1, v1, n, bits, s);
}

uint64_t unique_sorted(const uint32_t *a, uint64_t n, uint32_t *out, hipStream_t s) {
    if (!n) return 0;
    DevBuf pos((n + 1) * 4);
    hipLaunchKernelGGL(k_run_flags<uint32_t>, grid_n(n + 1), dim3(RBLK), 0, s, a, n, pos.u32());
    KETO_HIP(hipGetLastError());
    build::scan_excl(pos.u32(), n, s);
    hipLaunchKernelGGL(k_run_compact<uint32_t>, grid_n(n), dim3(RBLK), 0, s, a, n, pos.u32(), out);
    KETO_HIP(hipGetLastError());
    uint32_t m = 0;
    KETO_HIP(hipMemcpyAsync(&m, pos.u32() + n, 4, hipMemcpyDeviceToHost, s));
    KETO_HIP(hipStreamSynchronize(s));
    return m;
}

void run_flags(const uint64_t *a, uint64_t n, uint32_t *flag, hipStream_t s) {
    hipLaunchKernelGGL(k_run_flags<uint64_t>, grid_n(n + 1), dim3(RBLK), 0, s, a, n, flag);
    KETO_HIP(hipGetLastError());
}
void run_flags(const uint32_t *a, uint64_t n, uint32_t *flag, hipStream_t s) {
    hipLaunchKernelGGL(k_run_flags<uint32_t>, grid_n(n + 1), dim3(RBLK), 0, s, a, n, flag);
    KETO_HIP(hipGetLastError());
}

void sum_u32(const uint32_t *v, uint64_t n, unsigned long long *out, hipStream_t s) {
    KETO_HIP(hipMemsetAsync(out, 0, 8, s));
    if (n) hipLaunchKernelGGL(k_sum_u32, grid_n(n, 4096), dim3(RBLK), 0, s, v, n, out);
    KETO_HIP(hipGetLastError());
}

}  // namespace prim
}  // namespace keto
