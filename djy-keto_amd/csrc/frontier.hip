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

// The arena is cut into FR_SHARDS slices of `scap` goals; a block spawns into slice
// blockIdx % FR_SHARDS, so the allocation counters of a generation are FR_SHARDS addresses,
// not one (a single counter serialises every block's atomic: ~60M/s).  A generation is the
// union of one contiguous range per slice; slices stack their generations.
constexpr uint32_t FR_SHARDS = 64;
constexpr uint32_t GEN_STRIDE = MAX_GEN + 2;
// ctrl: gbase[FR_SHARDS][GEN_STRIDE] | gcount[FR_SHARDS][GEN_STRIDE] | fallback count (+3) |
// occurrence counts[FR_SHARDS]
constexpr size_t FR_CTRL_BYTES = (2 * FR_SHARDS * GEN_STRIDE + 4 + FR_SHARDS) * 4;

struct FrontierParams {
    DevSnapshot s;
    const uint4 *start;  // resolve records: 2 per query position (resolve.hip)
    uint32_t n;
    uint4 *g0;
    uint2 *gfn;
    uint2 *gvs;                  // {value, goals below (fr_reduce): the root's is the query's count}
    uint32_t cap, scap;          // arena goals, goals per slice
    uint32_t *gbase, *gcount;    // [FR_SHARDS][GEN_STRIDE]: slice-local base and count per generation
    uint32_t gen;
    uint32_t gen_cap;            // generations this batch may run (MAX_GEN; asynchronous batches: the speculated count)
    uint32_t *qrouted;           // [n / 32] one bit per query position: routed to the DFS interpreter (L2-resident)
    uint32_t *qspawn;            // [n] goals a query spawned from generation KETO_FR_CAP_GEN on (a lower bound)
    uint32_t *any_routed;        // != 0 once some query of the batch was routed (cleared with ctrl)
    uint32_t budget;
    unsigned long long *dkeys;   // decisive (scope, visited key) pairs of the batch (epoch-tagged)
    uint32_t *dcnt;              // their occurrences, counted by fr_repeat
    uint32_t *dbits;             // 2^DBITS_LOG2-bit filter of the decisive keys (L2-resident)
    uint32_t dmask, epoch;
    uint2 *occ;                  // every ES child's {scope, visited key}: FR_SHARDS slices of ocap
    uint32_t *occ_count;         // [FR_SHARDS] entries per slice
    uint32_t ocap;
    uint32_t max_width;
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t err_detail;
    uint32_t *fb_list, *fb_count;  // routed positions (+ pos_base: batch positions), for the DFS interpreter
    uint32_t pos_base;             // this pass's first batch position (batches of > FR_MAX_BATCH run in passes)
    unsigned long long *prof;      // KETO_FR_PROF builds: wave-cycles per phase of fr_expand
};

// Profiling builds (-DKETO_FR_PROF, tools/ab_build.sh): shader clock between phase marks
#ifdef KETO_FR_PROF
#define FR_MARK(n)                                                     \
    do {                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
        pacc[n] += t_ - pt;                                            \
        pt = t_;                                                       \
    } while (0)
#else
#define FR_MARK(n) ((void)0)
#endif

__device__ __forceinline__ Subject load_subject(const FrontierParams &P, uint32_t pos) {
    return subject_of(P.start[2 * (size_t)pos + 1]);  // one load
}
// Decisive-key table: keys carry the batch's epoch (1..TAB_EPOCHS) in bits 61-63 (scope < 2^29:
// a goal index), so the table is cleared once every TAB_EPOCHS batches instead of after each one:
// a slot holding 0 or another epoch's key is free.  Within a batch a slot only ever goes from
// free to a key of the batch, so a lookup may stop at the first free slot.
constexpr uint32_t TAB_EPOCHS = 7;
constexpr int TAB_PROBES = 256;  // a longer walk than this routes the query (crowded)
__device__ __forceinline__ unsigned long long tab_key(uint32_t ep, uint32_t scope, uint32_t vk) {
    return ((unsigned long long)ep << 61) | ((unsigned long long)scope << 32) | vk;
}
__device__ __forceinline__ bool tab_free(unsigned long long k, uint32_t ep) { return (uint32_t)(k >> 61) != ep; }
// insert `key` starting at slot h whose current content is `old` (the caller's first CAS of 0 ->
// key returned it); the slot where the key lives, -1 when the table is crowded.  *rep: the key
// was already there.
__device__ __forceinline__ int64_t tab_insert(unsigned long long *tk, uint32_t mask, uint32_t ep, unsigned long long key,
                                              uint32_t h, unsigned long long old, bool *rep) {
    *rep = false;
    for (int probe = 0; probe < TAB_PROBES;) {
        if (old == 0ull) return h;  // the CAS of 0 -> key that produced `old` inserted it
        if (old == key) {
            *rep = true;
            return h;
        }
        if (tab_free(old, ep)) {  // a stale key: replace it
            const unsigned long long r = atomicCAS(&tk[h], old, key);
            if (r == old) return h;
            old = r;  // another lane wrote a key of this batch here: look at it again
            continue;
        }
        h = (h + 1) & mask;
        probe++;
        old = atomicCAS(&tk[h], 0ull, key);
    }
    return -1;
}

__device__ __forceinline__ uint32_t tab_hash(unsigned long long key, uint32_t mask) {
    return (uint32_t)mix64(key & ((1ull << 61) - 1ull)) & mask;  // the epoch does not move a key
}
// The decisive keys' bit filter: fr_repeat looks up the table only for occurrences whose bit is
// set.  64 KB: every fr_repeat block holds it in LDS.  Decisive ES children are rare (Drive: ~3
// per 1000 queries), so nearly every occurrence is dismissed without a global access.
constexpr uint32_t DBITS_LOG2 = 19;
constexpr uint32_t REPEAT_BLOCK = 1024;
__device__ __forceinline__ uint32_t dbit(unsigned long long key) {
    return (uint32_t)(mix64(key & ((1ull << 61) - 1ull)) >> 40) & ((1u << DBITS_LOG2) - 1u);
}

// a routed query: its bit (every later goal of it stops spawning; generation 0 hands it over).
// One bit per query keeps the flags every goal reads in L2 (128 KB per 2^20 queries) instead of
// a 4-byte word per query that every goal fetched as a random line from HBM.
__device__ __forceinline__ void route(const FrontierParams &P, uint32_t pos) {
    atomicOr(&P.qrouted[pos >> 5], 1u << (pos & 31u));
    if (!*P.any_routed) atomicOr(P.any_routed, 1u);  // (rare: one word, written once per batch in practice)
}
__device__ __forceinline__ bool routed(const FrontierParams &P, uint32_t pos) { return (P.qrouted[pos >> 5] >> (pos & 31u)) & 1u; }

__device__ __forceinline__ void spawn(const FrontierParams &P, uint32_t c, uint32_t node, uint32_t pos, uint32_t word,
                                      uint32_t scope) {
    P.g0[c] = make_uint4(node, pos, word, scope);
}


// a generation's slices: exclusive prefix of their counts and their slice-local bases (LDS)
struct GenMap {
    uint32_t pre[FR_SHARDS + 1], base[FR_SHARDS];
};
__device__ __forceinline__ void load_gen(const FrontierParams &P, uint32_t k, GenMap &m) {
    for (uint32_t t = threadIdx.x; t < FR_SHARDS; t += blockDim.x) {
        const uint32_t b = P.gbase[t * GEN_STRIDE + k];
        m.base[t] = b;
        m.pre[t + 1] = std::min(P.gcount[t * GEN_STRIDE + k], P.scap - std::min(b, P.scap));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m.pre[0] = 0;
        for (uint32_t t = 0; t < FR_SHARDS; t++) m.pre[t + 1] += m.pre[t];
    }
    __syncthreads();
}
// the j-th goal of the generation (j < pre[FR_SHARDS]) -> arena index
__device__ __forceinline__ uint32_t gen_goal(const FrontierParams &P, const GenMap &m, uint32_t j) {
    uint32_t lo = 0, hi = FR_SHARDS;  // last slice with pre[t] <= j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (m.pre[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo * P.scap + m.base[lo] + (j - m.pre[lo]);
}

// the generation engine's sink: goal records into the arena, occurrences into the sliced list
struct GlobalSink {
    const FrontierParams &P;
    __device__ __forceinline__ void spawn(uint32_t c, uint32_t node, uint32_t pos, uint32_t word, uint32_t scope) const {
        LP(LP_WGOAL, &P.g0[c]);
        P.g0[c] = make_uint4(node, pos, word, scope);
    }
    __device__ __forceinline__ void spawn_es(uint32_t c, uint32_t node, uint32_t pos, uint32_t word, uint32_t scope,
                                             uint32_t) const {
        spawn(c, node, pos, word, scope);
    }
    __device__ __forceinline__ void occ(uint32_t o, uint32_t scope, uint32_t key) const {
        LP(LP_WOCC, &P.occ[o]);
        P.occ[o] = make_uint2(scope, key);
    }
};
// generation 0: query position i in slice i / chunk
__global__ __launch_bounds__(256) void fr_init(FrontierParams P) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t chunk = (P.n + FR_SHARDS - 1) / FR_SHARDS;
    if (i < FR_SHARDS) {
        P.gbase[i * GEN_STRIDE] = 0;
        P.gcount[i * GEN_STRIDE] = std::min(chunk, P.n - std::min(P.n, i * chunk));
    }
    if (i >= P.n) return;
    const uint4 r0 = P.start[2 * (size_t)i];
    const uint32_t d = r0.z & 0xFFFFu;
    P.g0[(i / chunk) * P.scap + i % chunk] = make_uint4(r0.x, i, gword(G_IA, d), NONE32);
    if (d > GD_MAX) route(P, i);  // (the bits were cleared before the launch)
    P.qspawn[i] = 0;
}

// One generation: every goal decides what it can and spawns its children into the next.
// Registers: 5 waves per SIMD (96 VGPRs).  Since the spine (frontier_goal.inc) the goal code
// holds more state; C4: 5 waves with phase B reloading the rewrite candidates' rows (no stash)
// 3.41 ms vs 6 waves with the stash 3.45 ms, 4 waves 3.59 ms (profiles/r04_waves_ab.txt).  (Round
// 2, before the spine: 6 waves 10.3 vs 5 waves 10.9 ms on the Drive profiling batch.)
#ifndef KETO_FR_WAVES
#define KETO_FR_WAVES 5
#endif
#ifndef KETO_FR_CAP_GEN
#define KETO_FR_CAP_GEN 8
#endif
#ifndef KETO_FR_BLOCK
#define KETO_FR_BLOCK 256
#endif
constexpr uint32_t XBLOCK = KETO_FR_BLOCK;  // fr_expand's block: the regroup window
template <bool LDS_TABLES>
__global__ __launch_bounds__(XBLOCK, KETO_FR_WAVES) void fr_expand(FrontierParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
    __shared__ GenMap gm;
    const uint32_t k = P.gen;
    load_gen(P, k, gm);
    const uint32_t cnt = gm.pre[FR_SHARDS];
    // the next generation in each slice starts where this one ends
    if (blockIdx.x == 0)
        for (uint32_t t = threadIdx.x; t < FR_SHARDS; t += blockDim.x)
            P.gbase[t * GEN_STRIDE + k + 1] = gm.base[t] + (gm.pre[t + 1] - gm.pre[t]);
    // blocks without a goal of this generation leave before staging the tables: small batches
    // and the empty generations an asynchronous batch launches speculatively cost ~nothing
    if (blockIdx.x * blockDim.x >= cnt) return;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    // A goal reads its query's routed bit only once some query of the batch was routed (by an
    // earlier generation, or this one so far): one word per block instead of a load per goal.
    // Routing is best-effort pruning here -- the decision at generation 0 reads the bits themselves.
#ifndef KETO_NO_RFLAG  // (A/B builds: every goal reads its bit)
    const bool any_routed = *P.any_routed != 0u;
#else
    const bool any_routed = true;
#endif
    // this wave's slice
    const uint32_t so = (blockIdx.x * ((blockDim.x + 63) >> 6) + (threadIdx.x >> 6)) % FR_SHARDS;
    const uint32_t nbase = so * P.scap + gm.base[so] + (gm.pre[so + 1] - gm.pre[so]), send = (so + 1) * P.scap;
    const bool last = k + 1 >= P.gen_cap;
    const uint32_t W = P.max_width;
#ifdef KETO_FR_PROF
    unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = __builtin_amdgcn_s_memtime();
#endif
#ifndef KETO_FR_RG_BUCKETS
#define KETO_FR_RG_BUCKETS 3
#endif
#ifndef KETO_FR_NOREGROUP
    constexpr uint32_t NB = KETO_FR_RG_BUCKETS;  // goal classes; dead lanes are one more
    __shared__ uint4 rg_g[XBLOCK];
    __shared__ uint32_t rg_i[XBLOCK], rg_n[XBLOCK / 64][NB + 1];
#ifndef KETO_FR_LATE_SUBJ
    __shared__ uint4 rg_s[XBLOCK];
#endif
#endif
    for (uint32_t j0 = blockIdx.x * blockDim.x; j0 < cnt; j0 += gridDim.x * blockDim.x) {
        const uint32_t j = j0 + threadIdx.x;
        // goals of queries routed meanwhile still run (rare); they can no longer spawn
        bool live = j < cnt;
        uint32_t i = live ? gen_goal(P, gm, j) : 0u;
#ifdef KETO_FR_LOADPROF
        if (live) LP(LP_G0, &P.g0[i]);
#endif
        uint4 g = live ? P.g0[i] : make_uint4(0, 0, 0, 0);
        // (the goal this thread loaded, and where the regroup put it: its gfn / gvs record is
        // written back by this thread, in generation order, from the slot's results)
        const bool own_live = live;
        const uint32_t own_i = i;
        uint32_t own_slot = threadIdx.x;
#if !defined(KETO_FR_NOREGROUP) && !defined(KETO_FR_LATE_SUBJ)
        // the query subject's membership record, loaded in generation order -- neighbouring goals
        // mostly belong to one query (a parent's children are contiguous), so a wave's loads fall
        // on few records and coalesce -- and carried through the regroup in LDS
#ifdef KETO_FR_LOADPROF
        if (live) LP(LP_SUBJ, &P.start[2 * (size_t)g.y + 1]);
#endif
        uint4 srec = live ? P.start[2 * (size_t)g.y + 1] : make_uint4(0, 0, 0, 0);
#endif
#ifndef KETO_FR_NOREGROUP
        {   // Block regroup: the block's goals ordered by class -- expand-subjects, rewrites, the
            // rest, then dead lanes; batch order within a class -- so that a wave runs one class's
            // code instead of several under divergence.
            const uint32_t wv = threadIdx.x >> 6, ln = __lane_id(), nw = (blockDim.x + 63) >> 6;
            uint32_t cls = NB;
            if (live) {
                const uint32_t kd = (g.z >> 12) & 7u;
                if (kd == G_ES) cls = 0;
                else if (NB > 2 && kd == G_RW) cls = 1;  // (an AND over one OR runs the OR's code: and_merge)
                else cls = NB - 1;
            }
            uint32_t rank = 0;
            for (uint32_t c = 0; c <= NB; c++) {
                const unsigned long long b = __ballot(cls == c);
                if (c == cls) rank = (uint32_t)__popcll(b & ((1ull << ln) - 1ull));
                if (ln == 0) rg_n[wv][c] = (uint32_t)__popcll(b);
            }
            __syncthreads();
            uint32_t slot = rank, n_live = 0;
            for (uint32_t c = 0; c <= NB; c++)
                for (uint32_t t = 0; t < nw; t++) {
                    const uint32_t m = rg_n[t][c];
                    if (c < cls || (c == cls && t < wv)) slot += m;
                    if (c < NB) n_live += m;
                }
            rg_g[slot] = g;
            rg_i[slot] = i;
#ifndef KETO_FR_LATE_SUBJ
            rg_s[slot] = srec;
#endif
            own_slot = slot;
            __syncthreads();
            g = rg_g[threadIdx.x];
            i = rg_i[threadIdx.x];
#ifndef KETO_FR_LATE_SUBJ
            srec = rg_s[threadIdx.x];
#endif
            live = threadIdx.x < n_live;
        }
#endif
        const uint32_t node = g.x, pos = g.y, w = g.z, scope = g.w;
        const uint32_t d = w & GD_MAX, kind = (w >> 12) & 7u, op = w >> 16;
        const bool qr = live && any_routed && routed(P, pos);
        // The loads the goal kinds start from, issued together: the row an ES / TTU reads, and
        // the subject's membership record (IA direct check, ES lookahead, OR shortcut).
        uint32_t rnode = NONE32;
        if (live && kind == G_ES && !(node & VIRT_BIT)) rnode = node;
        if (live && kind == G_TTU && d > 1) {
            const uint32_t ts = t_sibling(T, node, t_node_info(T, node), T.ops[op].rel_computed & 0xFFFFu);
            if (!(ts & VIRT_BIT)) rnode = ts;
        }
#ifdef KETO_FR_LOADPROF
        if (rnode != NONE32) LP(LP_ROW, &s.set_row[rnode]);
        if (live && any_routed) LP(LP_ROUTED, &P.qrouted[pos >> 5]);
#endif
        const uint4 row = rnode != NONE32 ? s.set_row[rnode] : make_uint4(0, 0, 0, 0);
#if !defined(KETO_FR_NOREGROUP) && !defined(KETO_FR_LATE_SUBJ)
        const Subject q = live ? subject_of(srec) : Subject{0, false, make_uint4(0, 0, 0, 0)};
#else
        const Subject q = live ? load_subject(P, pos) : Subject{0, false, make_uint4(0, 0, 0, 0)};
#endif
        FR_MARK(0);
        // ---- phase A: decide, or count the children -------------------------------------------
        const PhaseA pa = phase_a(s, T, q, live, node, w, scope, i, row, W);
        uint32_t nc = pa.nc, val = pa.val;
        const uint32_t rop = pa.rop, pat = pa.pat, sc = pa.sc, xrel = pa.xrel;
        const bool chain = pa.chain;
        (void)sc;
        if (nc > NC_MAX) {  // a row too long for the record: the DFS interpreter takes the query
            route(P, pos);
            nc = 0;
        }
        FR_MARK(1);
        // ---- budget and generation cap.  A query's goal count is its root's subtree count, summed
        // bottom-up by fr_reduce (gvs.y) without atomics, and compared with the budget at
        // generation 0; here a routed query (its bit set by route) stops spawning, as does
        // a goal with more children than the budget or at the last generation.  A query past its
        // budget spawns on meanwhile (bounded by MAX_GEN and its arena slice) -----------------------
        const uint32_t lane = __lane_id();
        if (nc && (qr || nc > P.budget || last)) {
            route(P, pos);
            nc = 0;
        }
#ifndef KETO_FR_NOSPAWNCAP  // (A/B builds only)
        // A query past its budget is routed at generation 0 anyway (fr_reduce's subtree count);
        // from generation KETO_FR_CAP_GEN on its spawns are also counted as they happen, and one
        // whose count alone passes the budget stops here: a runaway query would otherwise keep
        // spawning until MAX_GEN and fill its arena slice, routing its neighbours with it.  (The
        // count is a lower bound of the subtree count, so the routed set is unchanged.)
        if (nc && k >= KETO_FR_CAP_GEN && 1u + atomicAdd(&P.qspawn[pos], nc) + nc > P.budget) {
            route(P, pos);
            nc = 0;
        }
#endif
        FR_MARK(2);
        // ---- allocation: one atomic per wave, on the wave's slice counter -------------------------
        uint32_t wtot = 0;
        const uint32_t off = wave_excl(nc, wtot);
        uint32_t wbase = 0;
        if (lane == 0 && wtot) wbase = atomicAdd(&P.gcount[so * GEN_STRIDE + k + 1], wtot);
        const uint32_t cb = nbase + __shfl(wbase, 0) + off;
        if (nc && (uint64_t)cb + nc > send) {  // slice full: route; fill the allocated slots that exist
            route(P, pos);
            for (uint32_t c = cb; c < send && c < cb + nc; c++) spawn(P, c, 0, pos, gword(G_DEAD, 0), NONE32);
            nc = 0;
            val = M_NOT;
        }
#if !defined(KETO_FR_NOREGROUP) && !defined(KETO_FR_OLDGFN)  // (KETO_FR_OLDGFN: A/B builds)
        // the goal records go out in generation order: the regrouped lane leaves them in its LDS
        // slot (rg_g: this lane alone read it since the regroup), the thread that loaded the goal
        // writes them -- consecutive goals from consecutive lanes, whole lines per wave instead of
        // one scattered 8 B + 4 B write per goal (those were most of the kernel's write requests)
        if (live) rg_g[threadIdx.x] = make_uint4(cb, nc | (rop << 24) | (chain ? GFN_CHAIN : 0u), val, 0);
        __syncthreads();
        if (own_live) {
            LP(LP_WFN, &P.gfn[own_i]);
            LP(LP_WFN, &P.gvs[own_i]);
            const uint4 r = rg_g[own_slot];
            P.gfn[own_i] = make_uint2(r.x, r.y);
            reinterpret_cast<uint32_t *>(P.gvs)[2 * (size_t)own_i] = r.z;
        }
#else
        (void)own_live;
        (void)own_i;
        (void)own_slot;
        if (live) {
            P.gfn[i] = make_uint2(cb, nc | (rop << 24) | (chain ? GFN_CHAIN : 0u));
            reinterpret_cast<uint32_t *>(P.gvs)[2 * (size_t)i] = val;
        }
#endif
        // ---- occurrences: an ES goal's kept children, goals and leaves alike, are the keys it
        // adds to its scope (CheckAndAddVisited, engine.go:157-160): one run of its wave's slice
        const uint32_t nocc = (live && kind == G_ES && (nc || xrel)) ? pat + (chain ? 1u : 0u) : 0u;
        uint32_t otot = 0;
        const uint32_t ooff = wave_excl(nocc, otot);
        uint32_t obase = 0;
        if (lane == 0 && otot) obase = atomicAdd(&P.occ_count[so], otot);
        uint32_t oc = __shfl(obase, 0) + ooff;
        const bool occ_ok = (uint64_t)oc + nocc <= P.ocap;
        if (nocc && !occ_ok) {  // list full: the DFS interpreter takes the query; the allocated slots
            route(P, pos);      // that exist are cleared, so fr_repeat never counts an older batch's pair
            for (uint32_t e = oc; e < P.ocap && e < oc + nocc; e++) P.occ[(size_t)so * P.ocap + e] = make_uint2(NONE32, 0);
        }
        oc += so * P.ocap;
        FR_MARK(3);
        // ---- phase B: write the children (the same walk as phase A) -------------------------------
        if (nc || (kind == G_ES && xrel)) {
            GlobalSink gs{P};
            PhaseA pb = pa;
            pb.nc = nc;
            phase_b(s, T, q, node, pos, w, scope, row, pb, cb, oc, occ_ok, gs);
        }
        FR_MARK(4);
    }
#ifdef KETO_FR_PROF
    if (__lane_id() == 0)
        for (int n = 0; n < 7; n++) atomicAdd(&P.prof[n], pacc[n]);
#endif
}

// a decisive occurrence of (scope, key): into the decisive table and its bit filter
__device__ __forceinline__ void dec_insert(const FrontierParams &P, uint32_t scope, uint32_t vk, uint32_t pos) {
    const unsigned long long key = tab_key(P.epoch, scope, vk);
    const uint32_t h = tab_hash(key, P.dmask);
    bool rep = false;
    const int64_t at = tab_insert(P.dkeys, P.dmask, P.epoch, key, h, atomicCAS(&P.dkeys[h], 0ull, key), &rep);
    if (at < 0) route(P, pos);  // crowded: the DFS interpreter takes the query
    else if (!rep) P.dcnt[at] = 0;
    const uint32_t b = dbit(key);
    atomicOr(&P.dbits[b >> 5], 1u << (b & 31u));
}

// One generation, bottom-up: each goal reduces its children in add order (checkgroup H0,
// binop.go, rewrites.go:183-199); a decisive occurrence of a repeated scope key routes the
// query; generation 0 writes the decisions.  Every goal of the generation was expanded in
// this batch, so its children range is always this batch's.
__global__ __launch_bounds__(256) void fr_reduce(FrontierParams P) {
    const DevSnapshot &s = P.s;
    const uint32_t k = P.gen;
    __shared__ GenMap gm;
    load_gen(P, k, gm);
    const uint32_t cnt = gm.pre[FR_SHARDS];
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
        const uint32_t i = gen_goal(P, gm, j);
        const uint2 fn = P.gfn[i];
        uint32_t val = reinterpret_cast<const uint32_t *>(P.gvs)[2 * (size_t)i];
        const uint32_t nc = fn.y & NC_MAX, rop = (fn.y >> 24) & 3u;
        uint32_t sub = nc;  // goals below this one (the budget's count)
        if (nc) {
            uint32_t res = NONE32;
            auto fold = [&](const uint2 v) {  // every child's count; the fold up to its result
                sub += v.y;
                if (res != NONE32) return;
                const uint32_t cv = v.x;
                if (rop == R_FIRST || rop == R_FIRST_AND) {  // first Err / IsMember
                    if (decisive(cv)) res = cv;
                } else if (rop == R_AND) {  // AND: the first non-member, keeping its error
                    if ((cv >> 8) != 0 || (cv & 3u) != M_IS) res = (cv & ~3u) | M_NOT;
                } else {  // NOT swaps IsMember / NotMember, keeps Unknown and the error
                    const uint32_t m = cv & 3u;
                    res = m == M_IS ? ((cv & ~3u) | M_NOT) : (m == M_NOT ? ((cv & ~3u) | M_IS) : cv);
                }
            };
#ifdef KETO_FR_RED_SERIAL
            for (uint32_t c = fn.x; c < fn.x + nc; c++) fold(P.gvs[c]);
#else
            // the children's records four at a time, their loads issued together
            const uint32_t ce = fn.x + nc;
            for (uint32_t c0 = fn.x; c0 < ce; c0 += 4) {
                uint2 v[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) v[u] = c0 + u < ce ? P.gvs[c0 + u] : make_uint2(0, 0);
#pragma unroll
                for (uint32_t u = 0; u < 4; u++)
                    if (c0 + u < ce) fold(v[u]);
            }
#endif
            if (res == NONE32) res = val != NONE32 ? val : (rop == R_AND ? M_IS : M_NOT);
            if (rop == R_FIRST_AND) res = and_map(res);  // an AND over its merged OR
            val = res;
        }
        P.gvs[i] = make_uint2(val, sub);
        if (k > 0 && decisive(val)) {  // a decisive ES child: its key goes into the decisive table
            const uint4 g = P.g0[i];
            if ((((g.z >> 12) & 7u) == G_IA || ((g.z >> 12) & 7u) == G_ES) && (g.z & GF_ESCHILD))  // (RW / TTU / INV hold an op there)
                dec_insert(P, g.w, (g.z & GF_ALIAS) ? s.vkey[g.x] : g.x, g.y);
            if (fn.y & GFN_CHAIN) {  // the child whose expand-subject it ran is decisive too
                const uint32_t rawc = s.set_row[g.x].z, cc = rawc & s.edge_mask;
                dec_insert(P, g.w == NONE32 ? i : g.w, (rawc & EDGE_ALIAS) ? s.vkey[cc] : cc, g.y);
            }
        }
        if (k == 0) {  // generation 0: one goal per query position
            const uint32_t pos = P.g0[i].y;
            if (routed(P, pos) || 1u + sub > P.budget) {
                P.fb_list[atomicAdd(P.fb_count, 1u)] = P.pos_base + pos;
                continue;
            }
            const uint32_t q = P.start[2 * (size_t)pos].w;
            const uint32_t err = val >> 8;
            P.out_allowed[q] = (err == 0 && (val & 3u) == M_IS) ? 1 : 0;
            P.out_err[q] = (int32_t)(P.err_detail ? err : err & 0xFFu);
        }
    }
}

// After every generation above 0 is reduced: each occurrence of a decisive key counts itself;
// a second occurrence routes the query (the scope's first goal holds its position).
__global__ __launch_bounds__(REPEAT_BLOCK) void fr_repeat(FrontierParams P) {
    __shared__ uint32_t pre[FR_SHARDS + 1];
    __shared__ uint4 bits[(1u << DBITS_LOG2) / 128];
    for (uint32_t t = threadIdx.x; t < (1u << DBITS_LOG2) / 128; t += blockDim.x) bits[t] = reinterpret_cast<const uint4 *>(P.dbits)[t];
    for (uint32_t t = threadIdx.x; t < FR_SHARDS; t += blockDim.x) pre[t + 1] = std::min(P.occ_count[t], P.ocap);
    __syncthreads();
    if (threadIdx.x == 0) {
        pre[0] = 0;
        for (uint32_t t = 0; t < FR_SHARDS; t++) pre[t + 1] += pre[t];
    }
    __syncthreads();
    const uint32_t total = pre[FR_SHARDS];
    constexpr uint32_t U = 4;  // occurrences in flight per lane (the loop is latency-bound)
    const uint32_t G = gridDim.x * blockDim.x;
    for (uint32_t j0 = blockIdx.x * blockDim.x + threadIdx.x; j0 < total; j0 += U * G) {
        uint2 o[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t j = j0 + u * G;
            o[u] = make_uint2(NONE32, 0);
            if (j < total) {
                uint32_t lo = 0, hi = FR_SHARDS;  // last slice with pre[t] <= j
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pre[mid] <= j) lo = mid;
                    else hi = mid;
                }
                o[u] = P.occ[(size_t)lo * P.ocap + (j - pre[lo])];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            if (o[u].x == NONE32) continue;
            const unsigned long long key = tab_key(P.epoch, o[u].x, o[u].y);
            const uint32_t b = dbit(key);
            if (!((reinterpret_cast<const uint32_t *>(bits)[b >> 5] >> (b & 31u)) & 1u)) continue;  // not a decisive key
            uint32_t h = tab_hash(key, P.dmask);
            for (int probe = 0; probe < TAB_PROBES; probe++) {
                const unsigned long long kk = P.dkeys[h];
                if (kk == key) {
                    if (atomicAdd(&P.dcnt[h], 1u) >= 1u) route(P, P.g0[o[u].x].y);
                    break;
                }
                if (tab_free(kk, P.epoch)) break;
                h = (h + 1) & P.dmask;
            }
        }
    }
}

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
    const void *kx = lds_tables ? reinterpret_cast<const void *>(&fr_expand<true>) : reinterpret_cast<const void *>(&fr_expand<false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kx, XBLOCK, lds) != hipSuccess || per_cu <= 0) per_cu = 4;
    const dim3 eg(cus * (uint32_t)std::min(per_cu, (int)(2048 / XBLOCK))), xb(XBLOCK), eb(BLOCK);
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
            if (lds_tables) hipLaunchKernelGGL(fr_expand<true>, eg, xb, lds, st.stream, P);
            else hipLaunchKernelGGL(fr_expand<false>, eg, xb, 0, st.stream, P);
            KETO_HIP(hipGetLastError());
        }
        for (int32_t g = (int32_t)G - 1; g >= 0; g--) {
            P.gen = (uint32_t)g;
            if (g == 0) {
                hipLaunchKernelGGL(fr_repeat, dim3(cus * 2), dim3(REPEAT_BLOCK), 0, st.stream, P);
                KETO_HIP(hipGetLastError());
            }
            hipLaunchKernelGGL(fr_reduce, dim3(cus * KETO_FR_RGRID), eb, 0, st.stream, P);
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
    for (uint32_t k = 0; gens == 0;) {
        const uint32_t kend = std::min(k + (k == 0 ? std::max(CHUNK, f.last_gens + 1) : CHUNK), MAX_GEN);
        for (; k < kend; k++) {
            P.gen = k;
            if (lds_tables) hipLaunchKernelGGL(fr_expand<true>, eg, xb, lds, st.stream, P);
            else hipLaunchKernelGGL(fr_expand<false>, eg, xb, 0, st.stream, P);
            KETO_HIP(hipGetLastError());
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
        hipLaunchKernelGGL(fr_reduce, rg, eb, 0, st.stream, P);
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
