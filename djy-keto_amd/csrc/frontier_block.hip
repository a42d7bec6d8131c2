// gfx950 block frontier engine: the default Check path.
//
// The same breadth-first evaluation as frontier.hip -- a goal per reference step, evaluated
// without visited pruning (oracle/refsem.c "Frontier semantics"), the goals of a query reduced
// bottom-up in add order, queries whose answer could depend on pruning routed to the DFS
// interpreter -- with the bookkeeping kept on chip.  A persistent workgroup takes a chunk of
// BQ queries and runs all of their generations itself:
//   - the chunk's start records, goal counts and route flags live in LDS (no random loads of
//     per-query state per goal);
//   - a generation's goal records are written by their parents into an LDS buffer and read
//     from it by the next step (GCAP per generation; more spill to the chunk's pages);
//   - the reduction records (first child, children | reduce op, value, occurrences) go to
//     pages of a global pool owned by the workgroup, written and read back by the same CU;
//   - the visited-scope occurrences (ES children's keys) too: a scope belongs to one query, so
//     repeats are counted inside the chunk -- only when one of its ES children is decisive.
// No per-generation launch, no host read-back: one launch answers the batch, the DFS
// interpreter then takes the routed queries (their count stays on the device).
//
// Semantics are frontier_goal.inc's phase A / phase B, shared with frontier.hip; the goal
// counts, generation counts and routed queries equal the restatement's (rs_check_u) exactly as
// long as the goal and occurrence page pools last (a chunk that outgrows them routes its queries).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "device_common.hpp"

namespace keto {
namespace {

#include "frontier_goal.inc"

constexpr uint32_t BQ = 128;                   // queries per chunk
constexpr uint32_t BB = 256;                   // workgroup threads
constexpr uint32_t GCAP = 384;                 // goals of a generation held in LDS
constexpr uint32_t PG_LOG2 = 12, PG = 1u << PG_LOG2;  // goals per page
constexpr uint32_t MAX_PAGES = 64;             // a chunk's goal indices: < 2^18 (BQ x 2 x budget fits)
constexpr uint32_t OPG_LOG2 = 12, OPG = 1u << OPG_LOG2;  // occurrences per page
constexpr uint32_t MAX_OPAGES = 64;
constexpr uint32_t DEC_CAP = 128;              // decisive ES keys counted per pass of the repeat check
constexpr uint32_t SCOPE_BITS = 18;            // occurrence entry x = scope | chunk slot << SCOPE_BITS
constexpr uint32_t DEC_BIT = 0x80000000u;      // ... | DEC_BIT: a decisive occurrence, not yet counted
static_assert((((BQ - 1) << SCOPE_BITS) | ((1u << SCOPE_BITS) - 1)) < DEC_BIT, "occurrence entry bits");
constexpr uint32_t NB = 3;                     // regroup classes (ES, RW, the rest) + dead lanes

// one page of a chunk's goals (structure of arrays, 36 B per goal)
struct GoalPage {
    uint4 g0[PG];      // goal records of generations past GCAP goals
    uint32_t fc[PG];   // first child
    uint32_t ncw[PG];  // children | reduce op << 24 | GFN_CHAIN
    uint32_t val[PG];  // value (or the partial), then the reduced value
    uint32_t occ[PG];  // an ES child's own key: its occurrence, else NONE32
    uint32_t occ2[PG]; // a chain: the chained child's key's occurrence
};

struct BlockParams {
    DevSnapshot s;
    const uint4 *start;  // resolve records, 2 per batch position of this pass
    uint32_t n, cq, budget, max_width, err_detail, pos_base;  // cq: queries per chunk (<= BQ)
    uint32_t *ctrl;      // [0] chunk queue, [1] goal pages taken, [2] occurrence pages taken
    GoalPage *gpool;
    uint32_t gpool_cap;
    uint2 *opool;        // occurrence pages (OPG entries each)
    uint32_t opool_cap;
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *fb_list, *fb_count;   // routed batch positions, for the DFS interpreter
    unsigned long long *stats;      // [0] goals, [1] routed, [2] max generations, [3] chunks
    uint2 *stash;                   // phase A's children (frontier_goal.inc Stash), a column per lane; or null
    uint32_t stash_stride;
};

struct Chunk {  // LDS state of the workgroup's current chunk
    uint4 start[2 * BQ];
    uint32_t qcnt[BQ], qrt[BQ];
    uint4 gbuf[2][GCAP];
    uint32_t gs[MAX_GEN + 2];
    uint32_t pt[MAX_PAGES], opt[MAX_OPAGES];
    uint32_t npages, nopages, gnext, onext, ndec, pool_out, nq, chunk, gens;
    uint32_t dcnt[DEC_CAP];
    uint2 dkey[DEC_CAP];
};

__device__ __forceinline__ GoalPage &gpage(const BlockParams &P, const Chunk &C, uint32_t i) {
    return P.gpool[C.pt[i >> PG_LOG2]];
}
__device__ __forceinline__ uint2 &occ_at(const BlockParams &P, const Chunk &C, uint32_t o) {
    return P.opool[(size_t)C.opt[o >> OPG_LOG2] * OPG + (o & (OPG - 1))];
}

// goal records of generation k+1 (chunk-local index c = gs[k+1] + j): the LDS buffer, else a page
struct BlockSink {
    const BlockParams &P;
    Chunk &C;
    uint32_t k;
    __device__ __forceinline__ void put(uint32_t c, uint4 g, uint32_t occ) const {
        const uint32_t j = c - C.gs[k + 1];
        GoalPage &pg = gpage(P, C, c);
        if (j < GCAP) C.gbuf[(k + 1) & 1][j] = g;
        else pg.g0[c & (PG - 1)] = g;
        pg.occ[c & (PG - 1)] = occ;
    }
    __device__ __forceinline__ void spawn(uint32_t c, uint32_t node, uint32_t pos, uint32_t word, uint32_t scope) const {
        put(c, make_uint4(node, pos, word, scope), NONE32);
    }
    __device__ __forceinline__ void spawn_es(uint32_t c, uint32_t node, uint32_t pos, uint32_t word, uint32_t scope,
                                             uint32_t o) const {
        put(c, make_uint4(node, pos, word, scope), o);
    }
    __device__ __forceinline__ void occ(uint32_t o, uint32_t scope, uint32_t key) const {
        // (pos: the chunk slot of the goal whose walk writes it -- every scope belongs to one query)
        occ_at(P, C, o) = make_uint2(scope | (cur_slot << SCOPE_BITS), key);
    }
    uint32_t cur_slot;
};

__device__ __forceinline__ void route_slot(Chunk &C, uint32_t slot) { C.qrt[slot] = 1; }

// the pages backing goal indices [0, ng) and occurrences [0, no): taken from the pools by one
// thread between two barriers; a workgroup keeps its pages for its later chunks
__device__ __forceinline__ void back_pages(const BlockParams &P, Chunk &C, uint32_t ng, uint32_t no) {
    while (C.npages < MAX_PAGES && C.npages * PG < ng) {
        const uint32_t p = atomicAdd(&P.ctrl[1], 1u);
        if (p >= P.gpool_cap) break;  // pool exhausted: goals past the backed range are routed
        C.pt[C.npages++] = p;
    }
    while (C.nopages < MAX_OPAGES && C.nopages * OPG < no) {
        const uint32_t p = atomicAdd(&P.ctrl[2], 1u);
        if (p >= P.opool_cap) break;
        C.opt[C.nopages++] = p;
    }
}

// fold one goal's children in add order (checkgroup H0, binop.go, rewrites.go:183-199)
__device__ __forceinline__ uint32_t fold(const BlockParams &P, const Chunk &C, uint32_t fc, uint32_t ncw, uint32_t val) {
    const uint32_t nc = ncw & NC_MAX, rop = (ncw >> 24) & 3u;
    if (!nc) return val;
    uint32_t res = NONE32;
    for (uint32_t c = fc; c < fc + nc && res == NONE32; c++) {
        const uint32_t cv = gpage(P, C, c).val[c & (PG - 1)];
        if (rop == R_FIRST || rop == R_FIRST_AND) {  // first Err / IsMember
            if (decisive(cv)) res = cv;
        } else if (rop == R_AND) {  // AND: the first non-member, keeping its error
            if ((cv >> 8) != 0 || (cv & 3u) != M_IS) res = (cv & ~3u) | M_NOT;
        } else {  // NOT swaps IsMember / NotMember, keeps Unknown and the error
            const uint32_t m = cv & 3u;
            res = m == M_IS ? ((cv & ~3u) | M_NOT) : (m == M_NOT ? ((cv & ~3u) | M_IS) : cv);
        }
    }
    if (res == NONE32) res = val != NONE32 ? val : (rop == R_AND ? M_IS : M_NOT);
    if (rop == R_FIRST_AND) res = and_map(res);  // an AND over its merged OR
    return res;
}

// a decisive occurrence: marked in place (each goal marks its own entries); C.ndec says some are
__device__ __forceinline__ void add_dec(const BlockParams &P, Chunk &C, uint32_t o) {
    if (o == NONE32 || o >= C.nopages * OPG) return;
    occ_at(P, C, o).x |= DEC_BIT;
    C.ndec = 1;
}

// 4 waves per SIMD (108 VGPRs, 32 B of scratch; the 25 KB of LDS per workgroup caps it at 6
// anyway): round 5, C4 p99 of 64Ki batches 0.645 / 0.640 vs 0.663 / 0.658 ms at 5 (96 VGPRs,
// 64 B of scratch).  (Round 4, before the reachability tables: 5 waves 0.566 / 0.562 vs 0.583 /
// 0.586 ms at 6, profiles/r04_waves_ab.txt)
#ifndef KETO_FRB_WAVES
#define KETO_FRB_WAVES 4
#endif

template <bool LDS_TABLES>
__global__ __launch_bounds__(BB, KETO_FRB_WAVES) void fr_block(BlockParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    __shared__ Chunk C;
    __shared__ uint4 rg_g[BB];
    __shared__ uint32_t rg_i[BB], rg_n[BB / 64][NB + 1];
    const DevSnapshot &s = P.s;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const uint32_t tid = threadIdx.x, NT = blockDim.x, W = P.max_width;  // (NT: BB; 1 in the CPU emulation)
    if (tid == 0) {
        C.npages = 0;
        C.nopages = 0;
    }
    unsigned long long s_goals = 0, s_routed = 0;
    uint32_t s_gens = 0;
    for (;;) {
        if (tid == 0) C.chunk = atomicAdd(&P.ctrl[0], 1u);
        __syncthreads();
        const uint32_t c0 = C.chunk * P.cq;
        if (c0 >= P.n) break;
        const uint32_t nq = std::min(P.cq, P.n - c0);
        // generation 0: the chunk's queries
        for (uint32_t t = tid; t < nq; t += NT) {
            const uint4 r0 = P.start[2 * (size_t)(c0 + t)], r1 = P.start[2 * (size_t)(c0 + t) + 1];
            C.start[2 * t] = r0;
            C.start[2 * t + 1] = r1;
            const uint32_t d = r0.z & 0xFFFFu;
            C.qcnt[t] = 1;
            C.qrt[t] = d > GD_MAX ? 1u : 0u;  // deeper than a goal word holds: the interpreter
            C.gbuf[0][t] = make_uint4(r0.x, t, root_word(s, T, subject_of(r1), r0.x, d), NONE32);
        }
        if (tid == 0) {
            C.gs[0] = 0;
            C.gs[1] = nq;
            C.onext = 0;
            C.ndec = 0;
            back_pages(P, C, nq, 0);
        }
        __syncthreads();
        if (C.npages * PG < nq) {  // no page for the roots (pool exhausted): the interpreter takes the chunk
            for (uint32_t t = tid; t < nq; t += NT) route_slot(C, t);
            __syncthreads();
            if (tid == 0) C.gs[1] = 0;
            __syncthreads();
        }
        for (uint32_t t = tid; t < nq && t < C.npages * PG; t += NT) gpage(P, C, t).occ[t] = NONE32;
        // ---- expansion: generation k -> k + 1 until one is empty -----------------------------------
        uint32_t k = 0;
        for (;; k++) {
            const uint32_t gk = C.gs[k], cnt = C.gs[k + 1] - gk;
            if (cnt == 0) break;
            const uint32_t glim = C.npages * PG;  // (goals past the backed range were routed)
            __syncthreads();
            if (tid == 0) C.gnext = 0;
            __syncthreads();
            const bool last = k + 1 >= MAX_GEN;
            for (uint32_t j0 = 0; j0 < cnt; j0 += NT) {
                const uint32_t j = j0 + tid;
                bool live = j < cnt && gk + j < glim;
                uint32_t i = gk + j;
                uint4 g = make_uint4(0, 0, 0, 0);
                if (live) g = j < GCAP ? C.gbuf[k & 1][j] : gpage(P, C, i).g0[i & (PG - 1)];
                {   // regroup the step's goals by class (as fr_expand): a wave runs one class's code
                    const uint32_t wv = tid >> 6, ln = __lane_id(), nw = (NT + 63) / 64;
                    uint32_t cls = NB;
                    if (live) {
                        const uint32_t kd = (g.z >> 12) & 7u;
                        cls = kd == G_ES ? 0u : (kd == G_RW ? 1u : NB - 1);
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
                    __syncthreads();
                    g = rg_g[tid];
                    i = rg_i[tid];
                    live = tid < n_live;
                }
                const uint32_t node = g.x, pos = g.y, w = g.z, scope = g.w;
                const uint32_t d = w & GD_MAX, kind = (w >> 12) & 7u, op = w >> 16;
                uint32_t rnode = NONE32;
                if (live && kind == G_ES && !(node & VIRT_BIT)) rnode = node;
                if (live && kind == G_TTU && d > 1) {
                    const uint32_t ts = t_sibling(T, node, t_node_info(T, node), T.ops[op].rel_computed & 0xFFFFu);
                    if (!(ts & VIRT_BIT)) rnode = ts;
                }
                const uint4 row = rnode != NONE32 ? s.set_row[rnode] : make_uint4(0, 0, 0, 0);
                const uint4 rrec = (live && kind == G_ES) ? reach_record(s, T, node) : make_uint4(NONE32, NONE32, NONE32, 0);
                const Subject q = live ? subject_of(C.start[2 * pos + 1]) : Subject{0, false, make_uint4(0, 0, 0, 0)};
                Stash st{P.stash ? P.stash + (blockIdx.x * blockDim.x + tid) : nullptr, P.stash_stride, 0};
                const PhaseA pa = phase_a(s, T, q, live, node, w, scope, i, row, W, rrec, &st);
                uint32_t nc = pa.nc;
                // routing: a row too long for the record, a routed query, the generation cap, a goal
                // with more children than the budget, and the query's goal count past the budget
                if (nc && (nc > NC_MAX || C.qrt[pos] || last || nc > P.budget)) {
                    route_slot(C, pos);
                    nc = 0;
                }
                if (nc && atomicAdd(&C.qcnt[pos], nc) + nc > P.budget) {
                    route_slot(C, pos);
                    nc = 0;
                }
                // allocation: one LDS atomic per wave for the children, one for the occurrences
                uint32_t wtot = 0, otot = 0;
                const uint32_t off = wave_excl(nc, wtot);
                uint32_t wbase = 0;
                if (__lane_id() == 0 && wtot) wbase = atomicAdd(&C.gnext, wtot);
                uint32_t cb = C.gs[k + 1] + __shfl(wbase, 0) + off;
                const uint32_t nocc = (live && kind == G_ES && (nc || pa.xrel)) ? pa.pat + (pa.chain ? 1u : 0u) : 0u;
                const uint32_t ooff = wave_excl(nocc, otot);
                uint32_t obase = 0;
                if (__lane_id() == 0 && otot) obase = atomicAdd(&C.onext, otot);
                const uint32_t oc = __shfl(obase, 0) + ooff;
                __syncthreads();
                if (tid == 0) back_pages(P, C, C.gs[k + 1] + C.gnext, C.onext);
                __syncthreads();
                const uint32_t gback = C.npages * PG, oback = C.nopages * OPG;
                if (nc && cb + nc > gback) {  // past the backed goal range: routed, its slots dead
                    route_slot(C, pos);
                    for (uint32_t c = cb; c < gback && c < cb + nc; c++)
                        BlockSink{P, C, k, pos}.spawn(c, 0, pos, gword(G_DEAD, 0), NONE32);
                    nc = 0;
                }
                const bool occ_ok = oc + nocc <= oback;
                if (nocc && !occ_ok) {  // occurrence pages exhausted: routed; the backed slots cleared
                    route_slot(C, pos);
                    for (uint32_t e = oc; e < oback && e < oc + nocc; e++) occ_at(P, C, e) = make_uint2(NONE32, 0);
                }
                if (live && i < glim) {
                    GoalPage &pg = gpage(P, C, i);
                    const uint32_t li = i & (PG - 1);
                    pg.fc[li] = cb;
                    pg.ncw[li] = nc | (pa.rop << 24) | (pa.chain ? GFN_CHAIN : 0u);
                    pg.val[li] = pa.val;
                    pg.occ2[li] = (pa.chain && occ_ok) ? oc : NONE32;
                }
                const bool stashed = st.p && (kind == G_RW || kind == G_TTU) && st.n == pa.nc && nc <= FR_STASH_K;
                if (nc && stashed) {  // the children phase A kept (as fr_expand)
                    BlockSink sink{P, C, k, pos};
                    for (uint32_t j = 0; j < nc; j++) {
                        const uint2 v = st.p[(size_t)j * st.stride];
                        sink.spawn(cb + j, v.x, pos, v.y, scope);
                    }
                } else if (nc || (live && kind == G_ES && pa.xrel)) {
                    BlockSink sink{P, C, k, pos};
                    PhaseA pb = pa;
                    pb.nc = nc;
                    phase_b(s, T, q, node, pos, w, scope, row, pb, cb, oc, occ_ok, sink);
                }
            }
            __syncthreads();
            if (tid == 0) C.gs[k + 2] = C.gs[k + 1] + C.gnext;
            __syncthreads();
        }
        const uint32_t gens = k;  // generation `gens` is the first empty one
        // ---- reduction, deepest generation first ------------------------------------------------
        for (int32_t kk = (int32_t)gens - 1; kk >= 1; kk--) {
            const uint32_t gk = C.gs[kk], cnt = C.gs[kk + 1] - gk, glim = C.npages * PG;
            for (uint32_t j = tid; j < cnt; j += NT) {
                const uint32_t i = gk + j;
                if (i >= glim) continue;
                GoalPage &pg = gpage(P, C, i);
                const uint32_t li = i & (PG - 1), ncw = pg.ncw[li];
                const uint32_t v = fold(P, C, pg.fc[li], ncw, pg.val[li]);
                pg.val[li] = v;
                if (decisive(v)) {  // a decisive ES child: its key (and a chain's child's) is checked for repeats
                    add_dec(P, C, pg.occ[li]);
                    if (ncw & GFN_CHAIN) add_dec(P, C, pg.occ2[li]);
                }
            }
            __syncthreads();
        }
        // ---- repeats: a decisive key that its scope received more than once routes the query ---------
        // (in passes of up to DEC_CAP marked keys: any number of decisive occurrences is counted)
        if (C.ndec) {
            const uint32_t no = std::min(C.onext, C.nopages * OPG);
            for (;;) {
                __syncthreads();
                if (tid == 0) C.ndec = 0;
                __syncthreads();
                for (uint32_t o = tid; o < no; o += NT) {  // take up to DEC_CAP marked entries, unmarking them
                    const uint2 e = occ_at(P, C, o);
                    if (e.x == NONE32 || !(e.x & DEC_BIT)) continue;
                    const uint32_t d = atomicAdd(&C.ndec, 1u);
                    if (d >= DEC_CAP) continue;
                    C.dkey[d] = make_uint2(e.x & ~DEC_BIT, e.y);
                    C.dcnt[d] = 0;
                    occ_at(P, C, o).x = e.x & ~DEC_BIT;
                }
                __syncthreads();
                const uint32_t nd = C.ndec, ndec = std::min(nd, DEC_CAP);
                if (nd == 0) break;
                for (uint32_t o = tid; o < no; o += NT) {
                    const uint2 e = occ_at(P, C, o);
                    if (e.x == NONE32) continue;
                    const uint32_t x = e.x & ~DEC_BIT;
                    for (uint32_t d = 0; d < ndec; d++)
                        if (C.dkey[d].x == x && C.dkey[d].y == e.y) atomicAdd(&C.dcnt[d], 1u);
                }
                __syncthreads();
                for (uint32_t d = tid; d < ndec; d += NT)
                    if (C.dcnt[d] >= 2) route_slot(C, C.dkey[d].x >> SCOPE_BITS);
                if (nd <= DEC_CAP) break;
            }
            __syncthreads();
        }
        // ---- generation 0: the decisions ----------------------------------------------------------
        for (uint32_t t = tid; t < nq; t += NT) {
            const uint32_t bpos = P.pos_base + c0 + t;
            if (C.qrt[t]) {
                P.fb_list[atomicAdd(P.fb_count, 1u)] = bpos;
                s_routed++;
                continue;
            }
            GoalPage &pg = gpage(P, C, t);
            const uint32_t v = fold(P, C, pg.fc[t], pg.ncw[t], pg.val[t]);
            const uint32_t qi = C.start[2 * t].w;
            const uint32_t err = v >> 8;
            P.out_allowed[qi] = (err == 0 && (v & 3u) == M_IS) ? 1 : 0;
            P.out_err[qi] = (int32_t)(P.err_detail ? err : err & 0xFFu);
        }
        if (tid == 0) {
            s_goals += C.gs[gens];
            s_gens = std::max(s_gens, gens);
        }
        __syncthreads();
    }
    // per workgroup: its goals, routed queries, deepest chunk
    for (int off = 32; off > 0; off >>= 1) s_routed += __shfl_down(s_routed, off);
    if (__lane_id() == 0 && s_routed) atomicAdd(&P.stats[1], s_routed);
    if (tid == 0) {
        atomicAdd(&P.stats[0], s_goals);
        atomicMax(&P.stats[2], (unsigned long long)s_gens);
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// host

static size_t al256b(size_t b) { return (b + 255) / 256 * 256; }

uint32_t run_frontier_block(const Snapshot &s, Stream &st, const CheckLaunch &L, uint64_t pos_base) {
    FrontierBlockScratch &f = st.frontier_block;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? s.dev.lds_bytes : 0;
    const void *kf = lds_tables ? reinterpret_cast<const void *>(&fr_block<true>) : reinterpret_cast<const void *>(&fr_block<false>);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, BB, lds) != hipSuccess || per_cu <= 0) per_cu = 1;
    per_cu = std::min(per_cu, 8);
    // chunks of BQ queries; a batch too small to give every resident workgroup one gets smaller
    // chunks (down to 16 queries), so its generations spread over more CUs
    const uint64_t resident = (uint64_t)cus * per_cu;
    const uint32_t cq = (uint32_t)std::min<uint64_t>(BQ, std::max<uint64_t>(16, (L.n + resident - 1) / resident));
    const uint64_t chunks = (L.n + cq - 1) / cq;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(resident, chunks));
    // pools: a workgroup keeps the pages its largest chunk needed; an average chunk needs one goal
    // page and one occurrence page, a worst-case chunk 64 of each (routed past what is left)
    const uint32_t gcap = std::max<uint32_t>(2048, 4 * grid), ocap = gcap;
    if (!f.mem || f.gpool_cap < gcap) {
        if (f.mem) KETO_HIP(hipFree(f.mem));
        f.mem = nullptr;
        const size_t bytes = al256b(64) + al256b((size_t)gcap * sizeof(GoalPage)) + al256b((size_t)ocap * OPG * 8) + 256;
        KETO_HIP(hipMalloc(&f.mem, bytes));
        char *p = static_cast<char *>(f.mem);
        f.ctrl = reinterpret_cast<uint32_t *>(p);
        p += al256b(64);
        f.gpool = p;
        p += al256b((size_t)gcap * sizeof(GoalPage));
        f.opool = p;
        f.gpool_cap = gcap;
        f.opool_cap = ocap;
        if (!f.host) KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&f.host), 64, 0));
    }
    if (f.fb_cap < L.n) {  // routed batch positions (+ their count) for the DFS interpreter
        if (f.fb_list) KETO_HIP(hipFree(f.fb_list));
        f.fb_list = nullptr;
        uint64_t c = 1u << 16;
        while (c < L.n) c <<= 1;
        KETO_HIP(hipMalloc(&f.fb_list, (c + 64) * 4));
        f.fb_count = f.fb_list + c;
        f.fb_cap = c;
    }
    KETO_HIP(hipMemsetAsync(f.ctrl, 0, 64, st.stream));
    BlockParams P{};
    P.s = s.dev;
    P.start = st.resolved + 2 * pos_base;
    P.n = (uint32_t)L.n;
    P.cq = cq;
    P.budget = L.budget;
    P.max_width = (uint32_t)L.max_width;
    P.err_detail = L.err_detail;
    P.pos_base = (uint32_t)pos_base;
    P.ctrl = f.ctrl;
    P.gpool = static_cast<GoalPage *>(f.gpool);
    P.gpool_cap = f.gpool_cap;
    P.opool = static_cast<uint2 *>(f.opool);
    P.opool_cap = f.opool_cap;
    P.out_allowed = L.out_allowed;
    P.out_err = L.out_err;
    P.fb_list = f.fb_list;
    P.fb_count = f.fb_count;
    P.stats = reinterpret_cast<unsigned long long *>(f.ctrl + 4);
    P.stash = frontier_stash(st, cus);
    P.stash_stride = st.frontier.stash_stride;
    KETO_HIP(hipMemsetAsync(P.fb_count, 0, 4, st.stream));
    if (lds_tables) hipLaunchKernelGGL(fr_block<true>, dim3(grid), dim3(BB), lds, st.stream, P);
    else hipLaunchKernelGGL(fr_block<false>, dim3(grid), dim3(BB), 0, st.stream, P);
    KETO_HIP(hipGetLastError());
    if (L.async) {
        st.frontier.stats.async_batches++;
        return FR_ROUTED_ON_DEVICE;
    }
    KETO_HIP(hipMemcpyAsync(f.host, f.ctrl, 64, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(f.host + 12, P.fb_count, 4, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    const unsigned long long *stv = reinterpret_cast<const unsigned long long *>(f.host + 4);
    const uint32_t routed = f.host[12];
    keto_frontier_stats &fs = st.frontier.stats;
    fs.batches++;
    fs.queries += L.n;
    fs.routed += routed;
    fs.goals += stv[0];
    fs.generations += stv[2];
    fs.max_generations = std::max<uint64_t>(fs.max_generations, stv[2]);
    st.frontier.last_gens = (uint32_t)stv[2];
    static const bool verbose = getenv("KETO_FR_VERBOSE") != nullptr;
    if (verbose)
        fprintf(stderr, "[frontier block] n %llu goals %llu routed %u max generations %llu, goal pages %u, occurrence pages %u\n",
                (unsigned long long)L.n, stv[0], routed, stv[2], f.host[1], f.host[2]);
    return routed;
}

}  // namespace keto
