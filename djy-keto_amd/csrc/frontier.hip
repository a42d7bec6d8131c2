// gfx950 frontier engine for batched Check with OPL rewrites.
//
// The reference evaluates one Check as a recursion of goroutines, one SQL statement per hop
// (internal/check/{engine,rewrites,binop}.go).  Its answer depends on sibling order only
// through the visited set (engine.go:151-162, graph_utils.go:38-53): a child already marked
// in the scope is skipped.  Evaluated without that pruning the recursion is a pure function
// of the snapshot -- "U", oracle/refsem.c "Frontier semantics" -- and U equals the eager
// DFS (check.hip) on every query where no repeated key of a scope has a decisive occurrence
// (the proof is in refsem.c).  So U can be evaluated breadth-first, a goal per check:
//
//   generation k --fr_expand--> generation k+1 --...-->  (until a generation is empty)
//   generation k <--fr_reduce-- generation k+1 <--...    (first-decisive / AND / NOT, add order)
//
// Every goal is one lane: no per-query state machine, no divergence across interpreter
// states, no frame stack.  A goal reads what its hop needs (its row, the subject's probe),
// decides what it can on the spot (a direct tuple, the OR shortcut's IN query, the
// found-lookahead), and writes its children contiguously into the next generation.  A query
// whose answer could depend on visited pruning -- some (scope, visited key) of an ES child
// occurs more than once in the scope and one occurrence is decisive -- is routed to the DFS
// interpreter, as are queries that spawn more than `budget` goals, run past MAX_GEN
// generations or overflow the arena.  Repeats are found without hashing every occurrence:
// fr_expand appends each ES child's (scope, key) to an occurrence list (sequential writes),
// fr_reduce enters only the decisive ones into a small table, and fr_repeat counts the list's
// occurrences of those keys.
//
// Goal records (HBM, one arena per stream, structure of arrays; 32 bytes per goal):
//   g0[i]   = {node, query position, word, scope}   16 B, written by the parent at spawn
//   gfn[i]  = {first child, children | reduce op}    8 B, written by fr_expand
//   gvs[i]  = {value (or the partial fr_reduce folds), goals below it}  8 B, fr_expand (value),
//             then fr_reduce (both)
// word: bits 0-11 rest depth, 12-14 kind, 15 skip_direct, 16-31 rewrite op (RW / TTU / INV);
// an IA goal an ES spawned keeps bit 16 (its key is an occurrence of the scope) and bit 17 (the
// key is the node's visited alias).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_common.hpp"

namespace keto {
namespace {

#include "frontier_goal.inc"
#include "frontier_kernels.inc"

}  // namespace

// ---------------------------------------------------------------------------------------------
// host

static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

// Arena: 64 goals per query of the batch (C4 spawns 21, C2 6), or twice the stream's last batch if
// that was more; a slice that still fills routes its overflowing queries to the DFS interpreter.
// Occurrences (every kept child of an expand-subject, subject-id leaves included) outnumber goals
// on member-heavy rows: their list holds KETO_FR_OCC_PER_GOAL per goal (8 B each against a goal's
// 32 B).  (C4 at 64 goals per query with half as many occurrences routed 28 % of its queries.)
// KETO_FR_GOALS_PER_QUERY in the environment overrides the goal count: processes sharing one
// device (the eight ranks of tests/test_gpu_c5.py) hold less.
#ifndef KETO_FR_GOALS_PER_QUERY
#define KETO_FR_GOALS_PER_QUERY 64
#endif
#ifndef KETO_FR_OCC_PER_GOAL
#define KETO_FR_OCC_PER_GOAL 2
#endif

void ensure_frontier(FrontierScratch &f, uint64_t n) {
    // sized for the next power of two of the batch: a growing stream of batches reallocates (and
    // synchronises the device) O(log n) times, not at every new largest batch
    static const uint64_t per_query = [] {
        const char *e = getenv("KETO_FR_GOALS_PER_QUERY");
        return e ? std::max<uint64_t>(1, strtoull(e, nullptr, 10)) : (uint64_t)KETO_FR_GOALS_PER_QUERY;
    }();
    uint64_t np = 1;
    while (np < n) np <<= 1;
    n = std::min(np, FR_MAX_BATCH);
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>({n * per_query, 2ull * f.last_goals, 1u << 20}),
                                             1ull << 29) / FR_SHARDS *
                          FR_SHARDS;
    if (f.mem && f.cap >= want && f.ncap >= n) return;
    if (f.mem) KETO_HIP(hipFree(f.mem));
    f.mem = nullptr;
    const uint64_t cap = std::max<uint64_t>(want, f.cap);
    const uint64_t ncap = std::max<uint64_t>(n, f.ncap);
    // decisive-key table: a few decisive ES children per query at most in practice; a crowded
    // table routes (never seen); the occurrence list: half the arena's goal count
    uint64_t dcap = 1u << 16;
    while (dcap < 4 * ncap) dcap <<= 1;
    const uint64_t ocap = cap * KETO_FR_OCC_PER_GOAL / FR_SHARDS;  // per slice
    const size_t ctrl = al256(FR_CTRL_BYTES);
    const size_t bytes = ctrl + al256(ncap * 12) + al256(cap * 16) + al256(cap * 8) + al256(cap * 8) + al256(dcap * 12) +
                         al256(ocap * FR_SHARDS * 8) + (1u << DBITS_LOG2) / 8;
    KETO_HIP(hipMalloc(&f.mem, bytes));
    char *p = static_cast<char *>(f.mem);
    f.ctrl = reinterpret_cast<uint32_t *>(p);
    f.fb_count = f.ctrl + 2 * FR_SHARDS * GEN_STRIDE;
    f.occ_count = f.fb_count + 4;
    p += ctrl;
    f.qrouted = reinterpret_cast<uint32_t *>(p);
    f.qspawn = f.qrouted + ncap;  // (the bits take ncap / 32 words of the first ncap)
    f.fb_list = f.qrouted + 2 * ncap;
    p += al256(ncap * 12);
    f.g0 = reinterpret_cast<uint4 *>(p);
    p += al256(cap * 16);
    f.gfn = reinterpret_cast<uint2 *>(p);
    p += al256(cap * 8);
    f.gvs = reinterpret_cast<uint2 *>(p);
    p += al256(cap * 8);
    f.dkeys = reinterpret_cast<unsigned long long *>(p);
    f.dcnt = reinterpret_cast<uint32_t *>(f.dkeys + dcap);
    p += al256(dcap * 12);
    f.occ = reinterpret_cast<uint2 *>(p);
    p += al256(ocap * FR_SHARDS * 8);
    f.dbits = reinterpret_cast<uint32_t *>(p);
    // the table starts empty; batches tag their keys with an epoch (TAB_EPOCHS)
    KETO_HIP(hipMemset(f.dkeys, 0, dcap * 12));
    f.epoch = 1;
    KETO_HIP(hipDeviceSynchronize());
    f.cap = cap;
    f.ncap = ncap;
    f.dcap = dcap;
    f.ocap = ocap;
    if (!f.host_ctrl) KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&f.host_ctrl), FR_CTRL_BYTES, 0));
    if (!f.host_gens) KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&f.host_gens), 64, 0));
    if (!f.gens_ev) KETO_HIP(hipEventCreateWithFlags(&f.gens_ev, hipEventDisableTiming));
}

// An asynchronous pass's generation count, as the synchronous path computes it on the host:
// the first generation whose goals (summed over the slices, each clamped to its slice) are none;
// G when all G launched generations spawned (its deeper queries were routed).
static_assert(FR_SHARDS == 64, "fr_gens_used: one lane per slice in one wave");
__global__ __launch_bounds__(64) void fr_gens_used(const uint32_t *gbase, const uint32_t *gcount, uint32_t scap, uint32_t G,
                                                    uint32_t *out) {
    const uint32_t sh = threadIdx.x;  // one lane per slice (FR_SHARDS = 64)
    uint32_t gens = G;
    for (uint32_t g = 0; g <= G && g < GEN_STRIDE; g++) {
        const uint32_t b = gbase[sh * GEN_STRIDE + g], c = gcount[sh * GEN_STRIDE + g];
        const uint32_t t = std::min(c, scap - std::min(b, scap));
        if (!__ballot(t != 0)) {
            gens = g;
            break;
        }
    }
    if (sh == 0) *out = gens;
}

// The phase-A stash of the stream's frontier engines (frontier_goal.inc Stash): a column of
// FR_STASH_K entries per resident lane (at most 2048 per CU), shared by the generation and block
// engines (one stream runs one batch at a time); null with KETO_FR_NOSTASH (A/B: phase B walks
// every goal again)
uint2 *frontier_stash(Stream &st, uint32_t cus) {
    static const bool no_stash = getenv("KETO_FR_NOSTASH") != nullptr;
    if (no_stash) return nullptr;
    FrontierScratch &f = st.frontier;
    if (!f.stash || f.stash_stride < cus * 2048u) {
        if (f.stash) KETO_HIP(hipFree(f.stash));
        f.stash = nullptr;
        KETO_HIP(hipMalloc(&f.stash, (size_t)FR_STASH_K * cus * 2048u * sizeof(uint2)));
        f.stash_stride = cus * 2048u;
    }
    return f.stash;
}

uint32_t run_frontier(const Snapshot &s, Stream &st, const CheckLaunch &L, uint64_t pos_base) {
    FrontierScratch &f = st.frontier;
    if (L.n > FR_MAX_BATCH) throw Error(KETO_E_LIMIT, "frontier pass larger than FR_MAX_BATCH");
    ensure_frontier(f, L.n);
    const uint32_t cus = (uint32_t)num_cus(s.device);
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? s.dev.lds_bytes : 0;
    uint32_t *gbase = f.ctrl, *gcount = f.ctrl + FR_SHARDS * GEN_STRIDE, *fb_count = f.fb_count;
    KETO_HIP(hipMemsetAsync(f.ctrl, 0, FR_CTRL_BYTES, st.stream));
    KETO_HIP(hipMemsetAsync(f.dbits, 0, (1u << DBITS_LOG2) / 8, st.stream));
    KETO_HIP(hipMemsetAsync(f.qrouted, 0, (L.n + 31) / 32 * 4, st.stream));
    FrontierParams P{};
    P.s = s.dev;
    P.start = st.resolved + 2 * pos_base;
    P.pos_base = (uint32_t)pos_base;
    P.n = (uint32_t)L.n;
    P.g0 = f.g0;
    P.gfn = f.gfn;
    P.gvs = f.gvs;
    P.cap = (uint32_t)f.cap;
    P.scap = (uint32_t)(f.cap / FR_SHARDS);
    P.gbase = gbase;
    P.gcount = gcount;
    P.qrouted = f.qrouted;
    P.qspawn = f.qspawn;
    P.any_routed = fb_count + 1;
#ifdef KETO_FR_LOADPROF
    {
        unsigned long long *lc = st.counters;
        KETO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(lp_counts), &lc, sizeof(lc)));
    }
#endif
    P.budget = L.budget;
    P.dkeys = f.dkeys;
    P.dcnt = f.dcnt;
    P.dbits = f.dbits;
    P.dmask = (uint32_t)(f.dcap - 1);
    P.occ = f.occ;
    P.stash = frontier_stash(st, cus);
    P.stash_stride = f.stash_stride;
    P.occ_count = f.occ_count;
    P.ocap = (uint32_t)f.ocap;
    P.epoch = f.epoch;
    P.max_width = (uint32_t)L.max_width;
    P.out_allowed = L.out_allowed;
    P.out_err = L.out_err;
    P.err_detail = L.err_detail;
    P.fb_list = f.fb_list;
    P.fb_count = fb_count;
    P.prof = st.counters;
    P.gen_cap = MAX_GEN;
    constexpr uint32_t BLOCK = 256;
    hipLaunchKernelGGL(fr_init, dim3((uint32_t)((L.n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st.stream, P);
    KETO_HIP(hipGetLastError());
    // expansion: generations until one is empty; the slice counts are read back every CHUNK
    // a persistent grid: exactly the blocks that fit at once (a block waiting for a free slot would
    // run only after a resident one finished its whole share)
    int per_cu = 0;
    const void *kx = lds_tables ? reinterpret_cast<const void *>(&fr_expand<true, false>) : reinterpret_cast<const void *>(&fr_expand<false, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kx, XBLOCK, lds) != hipSuccess || per_cu <= 0) per_cu = 4;
    const dim3 eg(cus * (uint32_t)std::min(per_cu, (int)(2048 / XBLOCK))), xb(XBLOCK), eb(BLOCK);
    // generation 0 (the query roots) runs an instantiation of its own: KETO_FR_WAVES0 waves per SIMD
    // (KETO_FR_ROOT_KERNEL, A/B: also compiled for IA and RW goals only, KM_ROOT)
    static const bool root0 = getenv("KETO_FR_ROOT_KERNEL") != nullptr;
    int per_cu0 = 0;
    const void *kx0 = root0 ? (lds_tables ? reinterpret_cast<const void *>(&fr_expand<true, false, KM_ROOT, KETO_FR_WAVES0>)
                                          : reinterpret_cast<const void *>(&fr_expand<false, false, KM_ROOT, KETO_FR_WAVES0>))
                            : (lds_tables ? reinterpret_cast<const void *>(&fr_expand<true, false, KM_ALL, KETO_FR_WAVES0>)
                                          : reinterpret_cast<const void *>(&fr_expand<false, false, KM_ALL, KETO_FR_WAVES0>));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu0, kx0, XBLOCK, lds) != hipSuccess || per_cu0 <= 0) per_cu0 = per_cu;
    const dim3 eg0(cus * (uint32_t)std::min(per_cu0, (int)(2048 / XBLOCK)));
    auto launch_gen = [&](uint32_t k) {
        if (k == 0 && root0) {  // (round 6, C4 at 7 waves: 718 us against the generic kernel's 618 us)
            if (lds_tables) hipLaunchKernelGGL((fr_expand<true, false, KM_ROOT, KETO_FR_WAVES0>), eg0, xb, lds, st.stream, P);
            else hipLaunchKernelGGL((fr_expand<false, false, KM_ROOT, KETO_FR_WAVES0>), eg0, xb, 0, st.stream, P);
        } else if (k == 0) {
            if (lds_tables) hipLaunchKernelGGL((fr_expand<true, false, KM_ALL, KETO_FR_WAVES0>), eg0, xb, lds, st.stream, P);
            else hipLaunchKernelGGL((fr_expand<false, false, KM_ALL, KETO_FR_WAVES0>), eg0, xb, 0, st.stream, P);
        } else if (lds_tables) {
            hipLaunchKernelGGL((fr_expand<true, false>), eg, xb, lds, st.stream, P);
        } else {
            hipLaunchKernelGGL((fr_expand<false, false>), eg, xb, 0, st.stream, P);
        }
        KETO_HIP(hipGetLastError());
    };
    if (L.async) {
        // KETO_F_ASYNC: nothing comes back to the host.  The stream's last synchronous batch says
        // how deep a batch goes; G generations (a margin over it) are launched and each one whose
        // predecessor spawned nothing returns at once (its blocks leave before staging the
        // tables).  A query that would spawn past G is routed: the DFS interpreter, launched on
        // the device-side count, answers it.  So the answers are the synchronous path's; only a
        // deeper-than-speculated query costs the slower engine.
#ifndef KETO_FR_SPEC_MARGIN
#define KETO_FR_SPEC_MARGIN 2  // (4 and 8 reduce blocks per CU: 1 % slower per step on C4)
#endif
#ifndef KETO_FR_RGRID
#define KETO_FR_RGRID 4
#endif
        // (a stream with no history speculates 24; every empty generation still costs two launches)
        if (f.gens_pending && hipEventQuery(f.gens_ev) == hipSuccess) {  // an earlier async pass's depth
            f.last_gens = *f.host_gens;
            f.gens_pending = false;
        }
        const uint32_t G = std::min<uint32_t>(MAX_GEN, f.last_gens ? f.last_gens + KETO_FR_SPEC_MARGIN : 24);
        P.gen_cap = G;
        for (uint32_t k = 0; k < G; k++) {
            P.gen = k;
            launch_gen(k);
        }
        for (int32_t g = (int32_t)G - 1; g >= 0; g--) {
            P.gen = (uint32_t)g;
            if (g == 0) {
                hipLaunchKernelGGL(fr_repeat, dim3(cus * 2), dim3(REPEAT_BLOCK), 0, st.stream, P);
                KETO_HIP(hipGetLastError());
            }
            hipLaunchKernelGGL(fr_reduce<false>, dim3(cus * KETO_FR_RGRID), eb, 0, st.stream, P);
            KETO_HIP(hipGetLastError());
        }
        if (!f.gens_pending) {  // this pass's depth, for a later one (one read-back in flight at a time)
            hipLaunchKernelGGL(fr_gens_used, dim3(1), dim3(FR_SHARDS), 0, st.stream, gbase, gcount, P.scap, G, fb_count + 3);
            KETO_HIP(hipGetLastError());
            KETO_HIP(hipMemcpyAsync(f.host_gens, fb_count + 3, 4, hipMemcpyDeviceToHost, st.stream));
            KETO_HIP(hipEventRecord(f.gens_ev, st.stream));
            f.gens_pending = true;
        }
        if (++f.epoch > TAB_EPOCHS) {
            KETO_HIP(hipMemsetAsync(f.dkeys, 0, f.dcap * 12, st.stream));
            f.epoch = 1;
        }
        f.stats.async_batches++;
        return FR_ROUTED_ON_DEVICE;
    }
    constexpr uint32_t CHUNK = 12;
    uint32_t gens = 0;
    uint32_t *hc = f.host_ctrl;
    std::vector<uint64_t> tot(MAX_GEN + 1, 0);  // goals per generation
    const uint64_t scap = f.cap / FR_SHARDS;
    // the first read-back comes after as many generations as the stream's previous batch had (+1,
    // the empty one that ends it): a steady workload pays one host round trip per batch
    // KETO_FR_GENTIME (diagnostics): HIP events around every generation's expansion, printed per batch
    static const bool gentime = getenv("KETO_FR_GENTIME") != nullptr;
    std::vector<hipEvent_t> gev;
    for (uint32_t k = 0; gens == 0;) {
        const uint32_t kend = std::min(k + (k == 0 ? std::max(CHUNK, f.last_gens + 1) : CHUNK), MAX_GEN);
        for (; k < kend; k++) {
            P.gen = k;
            if (gentime) {
                gev.emplace_back();
                KETO_HIP(hipEventCreate(&gev.back()));
                KETO_HIP(hipEventRecord(gev.back(), st.stream));
            }
            launch_gen(k);
        }
        if (gentime) {
            gev.emplace_back();
            KETO_HIP(hipEventCreate(&gev.back()));
            KETO_HIP(hipEventRecord(gev.back(), st.stream));
        }
        KETO_HIP(hipMemcpyAsync(hc, f.ctrl, 2 * FR_SHARDS * GEN_STRIDE * 4, hipMemcpyDeviceToHost, st.stream));
        KETO_HIP(hipStreamSynchronize(st.stream));
        for (uint32_t g = 0; g <= k && g <= MAX_GEN; g++) {
            uint64_t t = 0;  // as fr_expand counts it: clamped to each slice
            for (uint32_t sh = 0; sh < FR_SHARDS; sh++) {
                const uint64_t b = hc[sh * GEN_STRIDE + g], c = hc[FR_SHARDS * GEN_STRIDE + sh * GEN_STRIDE + g];
                t += std::min<uint64_t>(c, scap - std::min<uint64_t>(b, scap));
            }
            tot[g] = t;
            if (t == 0) {
                gens = g;
                break;
            }
        }
        if (gens == 0 && k >= MAX_GEN) gens = MAX_GEN;  // the last generation spawned nothing (routed)
    }
    // reduction, deepest generation first
    uint64_t top = 0;
    for (int32_t g = (int32_t)gens - 1; g >= 0; g--) {
        top += tot[g];
        P.gen = (uint32_t)g;
        if (g == 0) {  // every decisive ES child is in the table: count the repeats of those keys
            hipLaunchKernelGGL(fr_repeat, dim3(cus * 2), dim3(REPEAT_BLOCK), 0, st.stream, P);
            KETO_HIP(hipGetLastError());
        }
        const dim3 rg((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((tot[g] + BLOCK - 1) / BLOCK, cus * 16)));
        hipLaunchKernelGGL(fr_reduce<false>, rg, eb, 0, st.stream, P);
        KETO_HIP(hipGetLastError());
    }
    if (++f.epoch > TAB_EPOCHS) {  // every TAB_EPOCHS batches: clear the table
        KETO_HIP(hipMemsetAsync(f.dkeys, 0, f.dcap * 12, st.stream));
        f.epoch = 1;
    }
    KETO_HIP(hipMemcpyAsync(hc, fb_count, 4, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    f.last_gens = gens;
    f.last_goals = (uint32_t)top;
    f.last_routed = hc[0];
    f.stats.batches++;
    f.stats.queries += L.n;
    f.stats.routed += hc[0];
    f.stats.goals += top;
    f.stats.generations += gens;
    f.stats.max_generations = std::max<uint64_t>(f.stats.max_generations, gens);
#if defined(KETO_FR_KINDSTAT) || defined(KETO_FR_LVSTAT)
    {
        unsigned long long ks[64 * 8];
        KETO_HIP(hipMemcpyFromSymbol(ks, HIP_SYMBOL(g_kstat), sizeof ks));
        static const unsigned long long zero[64 * 8] = {};
        KETO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_kstat), zero, sizeof zero));
        fprintf(stderr, "[kinds] n %llu:", (unsigned long long)L.n);
        for (uint32_t g = 0; g <= gens && g < 64; g++) {
            fprintf(stderr, " |");
            for (uint32_t kd = 0; kd < 8; kd++) fprintf(stderr, " %llu", ks[g * 8 + kd]);
        }
        fprintf(stderr, "\n");
    }
#endif
    if (gentime) {
        fprintf(stderr, "[gentime] n %llu us:", (unsigned long long)L.n);
        for (uint32_t g = 0; g + 1 < gev.size() && g <= gens; g++) {
            float ms = 0;
            KETO_HIP(hipEventElapsedTime(&ms, gev[g], gev[g + 1]));
            fprintf(stderr, " %.0f", ms * 1e3);
        }
        fprintf(stderr, "\n");
        for (hipEvent_t e : gev) KETO_HIP(hipEventDestroy(e));
    }
    static const bool verbose = getenv("KETO_FR_VERBOSE") != nullptr;
    if (verbose) {
        fprintf(stderr, "[frontier] n %llu generations %u goals %llu routed %u:", (unsigned long long)L.n, gens,
                (unsigned long long)top, hc[0]);
        for (uint32_t g = 0; g < gens; g++) fprintf(stderr, " %llu", (unsigned long long)tot[g]);
        fprintf(stderr, "\n");
    }
    return hc[0];
}

}  // namespace keto
