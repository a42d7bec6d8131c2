// gfx950 batched Check with OPL userset rewrites: exact one-worker sequential semantics.
//
// The reference evaluates one Check as a recursion of goroutines issuing one SQL
// statement per hop (internal/check/{engine,rewrites,binop}.go).  Here every lane of a
// persistent 64-wide wavefront owns one query and walks the same recursion as an explicit
// stack of 16-byte frames (checkIsAllowed, expandSubject, rewrite, shortcut candidates,
// tuple-to-userset, inverted).  The walk is cut into steps that need at most one dependent
// global round trip: every loop iteration each lane issues its (up to two, independent)
// 16-byte loads in the same instructions as every other lane, then consumes them with
// ALU/LDS work only.  Live state is kept in scalars (no runtime-indexed private arrays,
// no scratch spills) so the kernel keeps a high wave occupancy for latency hiding.
//
// Data placement: CSR rows, reverse rows and the probe hash in HBM (L2 / Infinity Cache
// resident when small); namespace table, relation info and rewrite program in LDS; the
// subject's reverse row in VGPRs when short (<= PROBE_K), else membership = one probe into
// the bucketized hash; per-lane visited sets (epoch-tagged, never cleared) and frame stacks
// in scratch.  Queries whose visited set or stack outgrow a tier are re-run by the next tier
// (bigger scratch, fewer lanes) through an on-device list: no host round trip in a batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.hpp"

namespace keto {
namespace {

constexpr uint32_t M_UNK = 0, M_IS = 1, M_NOT = 2;
__device__ __forceinline__ uint32_t mk_err(uint32_t e) { return e << 8; }
__device__ __forceinline__ bool decisive(uint32_t r) { return (r >> 8) != 0 || (r & 3u) == M_IS; }

// frame word w: bits 0-15 depth, 16-19 type, 20-23 phase, 24 skip_direct, 25 visited-scope owner
enum FrameType : uint32_t { F_IA = 0, F_ES = 1, F_RW = 2, F_SC = 3, F_TTU = 4, F_INV = 5 };
// FL_INLINE: S_FSCAN's window is the row descriptor's two inline edges (set by S_ROWOFF)
constexpr uint32_t FL_SKIP = 1u << 24, FL_OWNER = 1u << 25, FL_INLINE = 1u << 26;
__device__ __forceinline__ uint32_t fw(uint32_t type, uint32_t d, uint32_t phase = 0, uint32_t flags = 0) {
    return (d & 0xFFFFu) | (type << 16) | (phase << 20) | flags;
}
__device__ __forceinline__ uint32_t f_d(uint32_t w) { return w & 0xFFFFu; }
__device__ __forceinline__ uint32_t f_type(uint32_t w) { return (w >> 16) & 0xFu; }
__device__ __forceinline__ uint32_t f_phase(uint32_t w) { return (w >> 20) & 0xFu; }
__device__ __forceinline__ uint32_t set_phase(uint32_t w, uint32_t p) { return (w & ~(0xFu << 20)) | (p << 20); }

// ES child loop (oracle/refsem.c SCHED_EAGER): checkgroup's Add returns as soon as child k is
// handed to the group's consumer (concurrent_checkgroup.go:150-159), so engine.go:151-162 marks
// the following siblings -- up to the next one that was not visited -- before child k runs, and
// after a decisive child marks all the rest before its result is sent.  Phase-3 ES frames keep
// {x cursor, y end, z pending sibling (marked, not run yet; NONE32 = none)}; phase 4 = draining.
// lane states; "pseudo" states need no load and are run by the same step loop
enum State : uint32_t {
    S_IDLE = 0,
    S_START,    // start record of the resolve pre-pass (2 x 16 B)
    S_RUN,      // pseudo: execute / resume the top frame
    S_RET,      // pseudo: return `res` to the parent frame
    S_POP,      // parent frame
    S_DPROBE,   // probe-hash answer for checkDirect
    S_ROWOFF,   // {begin, end} of a subject-set row (ES or TTU)
    S_FSCAN,    // edge window of the ES found-lookahead
    S_FPROBE,   // probe-hash answers of the lookahead (<= 2)
    S_ESDONE,   // pseudo: lookahead exhausted -> truncate, open scope, child loop
    S_CNEXT,    // pseudo: ES child loop, next child
    S_CEDGE,    // edge window of the ES child loop
    S_VKEY,     // visited alias key
    S_VIS,      // visited slot pair
    S_TNEXT,    // pseudo: TTU loop, next parent
    S_TEDGE,    // edge window of the TTU loop
    S_SPROBE,   // probe-hash answers of the OR shortcut IN query (<= 2)
    S_CDISP,    // pseudo: the advance found the next unvisited sibling `cc` (NONE32: none left)
};

struct CheckParams {
    DevSnapshot s;
    const uint4 *start;     // resolve pre-pass records, in work order
    const uint32_t *qlist;  // tiers >= 1: start-record positions to (re)run
    const uint32_t *qlist_count;
    uint32_t n;
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *next;  // work-queue head
    uint32_t *ovf_list;
    uint32_t *ovf_count;
    unsigned long long *vis;  // [lanes * vcap]
    uint4 *stack;             // [lanes * scap]
    uint32_t *epochs;         // [lanes]
    uint32_t vcap, scap;
    int32_t max_depth, max_width;
    unsigned long long *counters;
    uint32_t last_tier;
    uint32_t live_lanes;  // lanes [live_lanes, 64) of every wave take no queries
    uint32_t err_detail;
};

#ifndef KETO_GUARD
#define KETO_GUARD 24
#endif
// Tier-0 resident blocks per CU (5 x 256 lanes = 5 waves per SIMD), below the 6 the register
// budget allows: fewer lanes, each running more queries, waste fewer lane-steps in the batch's
// tail.  C4 tier-0 kernel at 3 / 4 / 5 / 6 blocks per CU: 25.1 / 22.6 / 21.6 / 22.0 ms.
#ifndef KETO_T0_BLOCKS_PER_CU
#define KETO_T0_BLOCKS_PER_CU 5
#endif
// one-frame register cache of the stack top (0: every return reloads its parent frame)
#ifndef KETO_PCACHE
#define KETO_PCACHE 0
#endif
// Tier-0 visited slots per lane (two per 16-byte probe): ~500 nodes per query scope
#ifndef KETO_T0_VCAP
#define KETO_T0_VCAP 1024
#endif

__device__ __forceinline__ uint32_t w8(const uint4 &v0, const uint4 &v1, uint32_t j) {
    return j < 4 ? wword(v0, j) : wword(v1, j - 4);
}
// one probe bucket: 1 found, 0 absent, 2 continue with the next bucket
__device__ __forceinline__ uint32_t probe_check(const uint4 &b, uint64_t key) {
    const uint64_t k0 = (uint64_t)b.x | ((uint64_t)b.y << 32), k1 = (uint64_t)b.z | ((uint64_t)b.w << 32);
    if (k0 == key || k1 == key) return 1;
    if (k0 == 0 || k1 == 0) return 0;
    return 2;
}

template <bool COUNT, bool LDS_TABLES>
__global__ __launch_bounds__(256) void check_kernel(CheckParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
#ifndef KETO_DFS_OLD
    // an empty device list (the frontier routed nothing, or no query outgrew the previous tier):
    // the whole block leaves before staging the tables (the value is the same for every thread)
    if (P.qlist && *P.qlist_count == 0) return;
#endif
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t pmask = (P.vcap >> 1) - 1;
    const uint32_t W = (uint32_t)P.max_width;
    const uint32_t lane = __lane_id();

    uint32_t q = 0, pos = 0, st = S_IDLE;
    bool exhausted = lane >= P.live_lanes;
    uint32_t sidx = NONE32;  // subject
    bool heavy = false;
    uint32_t R0 = NONE32, R1 = NONE32, R2 = NONE32, R3 = NONE32;
    // interpreter
    uint4 top = make_uint4(0, 0, 0, 0);
    // one-frame register cache of the stack top (write-back): a call's frame is written to the
    // scratch stack only when a deeper call evicts it, so a leaf call + return costs no memory
    uint4 pcache = make_uint4(0, 0, 0, 0);
    bool pc_ok = false;
    uint32_t sp = 0, res = 0, vcount = 0;
    bool have_res = false, scope = false;
    uint4 ew = make_uint4(0, 0, 0, 0);
    uint32_t ew_lo = 1, ew_hi = 0;      // edge indices present in ew
    uint32_t aux = 0, aux2 = 0;         // probe buckets / visited pair
    uint32_t pc0 = 0, pc1 = 0, pn = 0;  // probed nodes, count
    uint32_t cc = 0, vk = 0;            // child node / its visited key
    const uint4 *la0 = nullptr, *la1 = nullptr;
    uint32_t ln = 0;
    uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
    unsigned long long c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0, c_wsteps = 0, c_lsteps = 0;

    while (true) {
        // ---- refill idle lanes: one atomic per wavefront (ballot + mbcnt) --------------------
        const bool need = (st == S_IDLE) && !exhausted;
        const unsigned long long mask = __ballot(need);
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(P.next, (uint32_t)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t my = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                if (my >= nq) exhausted = true;
                else {
                    pos = P.qlist ? P.qlist[my] : my;
                    st = S_START;
                    la0 = P.start + 2 * (size_t)pos;
                    la1 = la0 + 1;
                    ln = 2;
                    q_rows = q_edges = q_probes = 0;
                }
            }
        }
        if (__ballot(st != S_IDLE) == 0) break;
        // ---- the load slot: every lane's loads in the same instructions ------------------------
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        if (ln > 0) v0 = *la0;
        if (ln > 1) v1 = *la1;
        ln = 0;
        if (COUNT) {
            c_wsteps += lane == 0 ? 1 : 0;
            c_lsteps += st != S_IDLE ? 1 : 0;
        }
        if (st == S_IDLE) continue;
#ifdef KETO_EMU_SKIP  // CPU-emulation builds only: the round-1 waterfall variant's unserved lanes
        // (a lane sits out the step after its operands were loaded; they are gone next step)
        if (mix64(((uint64_t)gl << 32) ^ (c_wsteps++ * 0x9E3779B97F4A7C15ull)) % KETO_EMU_SKIP == 0) continue;
#endif
#ifdef KETO_EMU_TRACE
        keto_emu_trace_step(st == S_START ? pos : NONE32);
#endif

#include "check_step.inc"
    }
    P.epochs[gl] = epoch;
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            c_rows += __shfl_down(c_rows, off);
            c_edges += __shfl_down(c_edges, off);
            c_probes += __shfl_down(c_probes, off);
            c_q += __shfl_down(c_q, off);
            c_lsteps += __shfl_down(c_lsteps, off);
        }
        if (lane == 0) {
            atomicAdd(&P.counters[0], c_rows);
            atomicAdd(&P.counters[1], c_edges);
            atomicAdd(&P.counters[2], c_probes);
            atomicAdd(&P.counters[4], c_q);
            atomicAdd(&P.counters[5], c_wsteps);
            atomicAdd(&P.counters[6], c_lsteps);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Block-regrouped interpreter (tier 0 of large batches).
//
// A wave-step costs one pass over every distinct case body its 64 lanes are in, and lanes that
// each own one query sit in ~20 different bodies per step.  Here a block's
// queries live in LDS slots instead of lanes: every step, each lane loads the slot it was dealt,
// issues the slot's load, runs the same transitions as check_kernel (check_step.inc), stores
// the slot back, and then the block counting-sorts its slots by the dispatch key they stopped
// at -- so at the next step the lanes of one wave hold queries in the same few states.
// tools/sim_regroup.py (CPU-emulation traces of the Drive workload) puts the case bodies per
// lane-step at 1.8x (256 slots) to 2.5x (1024 slots) fewer.  Visited tables, frame stacks and
// epochs belong to the slot, so a query may run on a different lane every step.
#ifndef KETO_RG_BLOCK
#define KETO_RG_BLOCK 512
#endif
#ifndef KETO_RG_MAX_BLOCKS_PER_CU  // resident blocks per CU (LDS-bound below this)
#define KETO_RG_MAX_BLOCKS_PER_CU 8
#endif
constexpr uint32_t RG = KETO_RG_BLOCK;
constexpr uint32_t RG_KEYS = 64;
constexpr uint32_t RG_GROUPS = 8 + KETO_PCACHE;  // 16-byte state groups per slot (+1 with work counting)

__host__ __device__ constexpr size_t rg_state_bytes(bool count) { return (size_t)RG * 16 * (RG_GROUPS + (count ? 1 : 0)); }
__host__ __device__ constexpr size_t rg_extra_bytes() { return (size_t)RG * 4 + 2 * RG_KEYS * 4 + 16; }

__device__ __forceinline__ uint32_t rg_key(uint32_t st, uint32_t w) {
    if (st != S_RUN) return st;  // S_IDLE = 0 sorts first: the lanes that refill are contiguous
    const uint32_t ph = f_phase(w) < 3 ? f_phase(w) : 3u;
    return 32 + f_type(w) * 4 + ph;
}

template <bool COUNT, bool LDS_TABLES>
__global__ __launch_bounds__(RG) void check_kernel_rg(CheckParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const size_t tab = LDS_TABLES ? ((size_t)s.lds_bytes + 15) / 16 * 16 : 0;
    uint4 *G = reinterpret_cast<uint4 *>(lds + tab);  // group g of slot k at G[g * RG + k]
    uint16_t *perm = reinterpret_cast<uint16_t *>(lds + tab + rg_state_bytes(COUNT));  // [2][RG]: lane -> slot
    uint32_t *hist = reinterpret_cast<uint32_t *>(perm + 2 * RG);                    // [2][RG_KEYS]
    uint32_t *flags = hist + 2 * RG_KEYS;  // [0] queue exhausted
    const uint32_t tid = threadIdx.x;
    const uint32_t base = blockIdx.x * RG;
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t pmask = (P.vcap >> 1) - 1;
    const uint32_t W = (uint32_t)P.max_width;
    const uint32_t lane = __lane_id();
    unsigned long long c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0, c_wsteps = 0, c_lsteps = 0;

    // every slot starts idle, with its epoch
    G[0 * RG + tid] = make_uint4(0, 0, 0, 0);
    G[1 * RG + tid] = make_uint4(0, 0, 0, 0);
    G[2 * RG + tid] = make_uint4(0, 0, NONE32, S_IDLE);
    G[3 * RG + tid] = make_uint4(NONE32, NONE32, NONE32, NONE32);
    G[4 * RG + tid] = make_uint4(0, 0, P.epochs[base + tid], 0);
    G[5 * RG + tid] = make_uint4(1, 0, 0, 0);
    G[6 * RG + tid] = make_uint4(0, 0, 0, 0);
    G[7 * RG + tid] = make_uint4(0, 0, 0, 0);
    if (KETO_PCACHE) G[8 * RG + tid] = make_uint4(0, 0, 0, 0);
    if (COUNT) G[RG_GROUPS * RG + tid] = make_uint4(0, 0, 0, 0);
    perm[tid] = (uint16_t)tid;
    if (tid < 2 * RG_KEYS) hist[tid] = 0;
    if (tid < 4) flags[tid] = 0;
    __syncthreads();
    uint32_t cur = 0;
    for (;;) {
        const uint32_t slot = perm[cur * RG + tid];
        unsigned long long *vis = P.vis + (size_t)(base + slot) * P.vcap;
        uint4 *stk = P.stack + (size_t)(base + slot) * P.scap;
        // ---- the slot's query state
        uint4 top = G[0 * RG + slot];
        uint4 ew = G[1 * RG + slot];
        const uint4 g2 = G[2 * RG + slot], g3 = G[3 * RG + slot], g4 = G[4 * RG + slot], g5 = G[5 * RG + slot],
                    g6 = G[6 * RG + slot], g7 = G[7 * RG + slot];
        uint32_t q = g2.x, pos = g2.y, sidx = g2.z;
        uint32_t st = g2.w & 63u, pn = (g2.w >> 9) & 3u, ln = (g2.w >> 11) & 3u;
        bool heavy = (g2.w >> 6) & 1u, have_res = (g2.w >> 7) & 1u, scope = (g2.w >> 8) & 1u;
        bool pc_ok = KETO_PCACHE && ((g2.w >> 13) & 1u);
        uint4 pcache = KETO_PCACHE ? G[8 * RG + slot] : make_uint4(0, 0, 0, 0);
        uint32_t R0 = g3.x, R1 = g3.y, R2 = g3.z, R3 = g3.w;
        uint32_t res = g4.x, vcount = g4.y, epoch = g4.z, sp = g4.w;
        uint32_t ew_lo = g5.x, ew_hi = g5.y, aux = g5.z, aux2 = g5.w;
        uint32_t cc = g6.x, vk = g6.y, pc0 = g6.z, pc1 = g6.w;
        const uint4 *la0 = reinterpret_cast<const uint4 *>((uintptr_t)g7.x | ((uintptr_t)g7.y << 32));
        const uint4 *la1 = reinterpret_cast<const uint4 *>((uintptr_t)g7.z | ((uintptr_t)g7.w << 32));
        uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
        if (COUNT) {
            const uint4 g9 = G[RG_GROUPS * RG + slot];
            q_rows = g9.x;
            q_edges = g9.y;
            q_probes = g9.z;
        }
        // ---- refill idle slots: one atomic per wavefront (ballot + mbcnt)
        const bool need = (st == S_IDLE) && flags[0] == 0;
        const unsigned long long mask = __ballot(need);
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            uint32_t b0 = 0;
            if ((int)lane == leader) b0 = atomicAdd(P.next, (uint32_t)__popcll(mask));
            b0 = __shfl(b0, leader);
            if (need) {
                const uint32_t my = b0 + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                if (my >= nq) flags[0] = 1;
                else {
                    pos = P.qlist ? P.qlist[my] : my;
                    st = S_START;
                    la0 = P.start + 2 * (size_t)pos;
                    la1 = la0 + 1;
                    ln = 2;
                    q_rows = q_edges = q_probes = 0;
                }
            }
        }
        // ---- the load slot, then the transitions (the same state machine as check_kernel)
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        if (ln > 0) v0 = *la0;
        if (ln > 1) v1 = *la1;
        ln = 0;
        if (COUNT) {
            c_wsteps += lane == 0 ? 1 : 0;
            c_lsteps += st != S_IDLE ? 1 : 0;
        }
        if (st != S_IDLE) {
#include "check_step.inc"
        }
        // ---- store the slot back
        G[0 * RG + slot] = top;
        G[1 * RG + slot] = ew;
        G[2 * RG + slot] = make_uint4(q, pos, sidx, st | (uint32_t(heavy) << 6) | (uint32_t(have_res) << 7) |
                                                         (uint32_t(scope) << 8) | (pn << 9) | (ln << 11) |
                                                         (uint32_t(pc_ok) << 13));
        G[3 * RG + slot] = make_uint4(R0, R1, R2, R3);
        G[4 * RG + slot] = make_uint4(res, vcount, epoch, sp);
        G[5 * RG + slot] = make_uint4(ew_lo, ew_hi, aux, aux2);
        G[6 * RG + slot] = make_uint4(cc, vk, pc0, pc1);
        G[7 * RG + slot] = make_uint4((uint32_t)(uintptr_t)la0, (uint32_t)((uintptr_t)la0 >> 32), (uint32_t)(uintptr_t)la1,
                                      (uint32_t)((uintptr_t)la1 >> 32));
        if (KETO_PCACHE) G[8 * RG + slot] = pcache;
        if (COUNT) G[RG_GROUPS * RG + slot] = make_uint4(q_rows, q_edges, q_probes, 0);
        // ---- regroup: counting sort of the slots by the key they stopped at (two barriers)
        const uint32_t key = rg_key(st, top.w);
        const uint32_t rank = atomicAdd(&hist[cur * RG_KEYS + key], 1u);
        if (tid < RG_KEYS) hist[(cur ^ 1) * RG_KEYS + tid] = 0;  // the next step's histogram
        __syncthreads();
        uint32_t pre = 0;  // slots in smaller keys: the histogram read 4 keys per load
        const uint4 *h4 = reinterpret_cast<const uint4 *>(hist + cur * RG_KEYS);
        for (uint32_t k4 = 0; k4 < RG_KEYS / 4; k4++) {
            const uint4 h = h4[k4];
            const uint32_t k = 4 * k4;
            pre += (k < key ? h.x : 0u) + (k + 1 < key ? h.y : 0u) + (k + 2 < key ? h.z : 0u) + (k + 3 < key ? h.w : 0u);
        }
        perm[(cur ^ 1) * RG + pre + rank] = (uint16_t)slot;
        const bool done = hist[cur * RG_KEYS] == RG && flags[0] != 0;  // every slot idle, queue drained
        __syncthreads();
        if (done) break;
        cur ^= 1;
    }
    P.epochs[base + tid] = G[4 * RG + tid].z;
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            c_rows += __shfl_down(c_rows, off);
            c_edges += __shfl_down(c_edges, off);
            c_probes += __shfl_down(c_probes, off);
            c_q += __shfl_down(c_q, off);
            c_lsteps += __shfl_down(c_lsteps, off);
        }
        if (lane == 0) {
            atomicAdd(&P.counters[0], c_rows);
            atomicAdd(&P.counters[1], c_edges);
            atomicAdd(&P.counters[2], c_probes);
            atomicAdd(&P.counters[4], c_q);
            atomicAdd(&P.counters[5], c_wsteps);
            atomicAdd(&P.counters[6], c_lsteps);
        }
    }
}

}  // namespace

// --------------------------------------------------------------------------------------
// host launcher

// The DFS interpreter over the resolved batch, or over the `nl` positions of the device list
// `list` (queries the frontier engine routed here).  Tier 0's kernel is timed when `timed`.
static void run_dfs(const Snapshot &s, Stream &st, const CheckLaunch &L, const uint32_t *list, const uint32_t *list_count,
                    uint64_t nl, bool timed, bool count_on_device = false) {
    constexpr uint32_t BLOCK = 256;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    // Queries that outgrow a tier's scratch go to the next (lanes, visited slots per lane,
    // frames per lane); HBM is plentiful (288 GB): tier 0 holds ~500 visited nodes per lane,
    // tier 1 ~4k, tier 2 ~500k.
    // Tier 0 is sized to the persistent grid it can ever launch (KETO_T0_BLOCKS_PER_CU resident
    // blocks per CU): 1.3k lanes x 9 KiB per CU, ~3 GiB per stream on 256 CUs.
    const Tier t[3] = {Tier{cus * KETO_T0_BLOCKS_PER_CU * 256, KETO_T0_VCAP, 64},  // the common case
                       Tier{cus * 64, 1u << 13, 1024},                      // wide visited scopes
                       Tier{64, 1u << 20, 1u << 14}};   // huge scopes / deep recursion
    ensure_scratch(st.check_scratch, t);
    Scratch &sc = st.check_scratch;
    uint32_t *lists[2] = {st.lists, st.lists + st.list_cap};
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? s.dev.lds_bytes : 0;
    KETO_HIP(hipMemsetAsync(sc.ctrl, 0, 64, st.stream));
    // The block-regrouped interpreter is opt-in: it halves the issued instructions on C4 but
    // measured 7-23% slower than the lane kernel on MI355X (every step ends
    // in a block barrier, which exposes the memory latency the lane kernel hides across waves).
    // KETO_REGROUP=1 uses it for batches that fill the resident blocks several times over,
    // =force for every batch (tests).
#ifdef KETO_CPUEMU
    const bool rg_on = false, rg_force = false;  // the CPU emulation runs one-lane waves
#else
    const char *rge = getenv("KETO_REGROUP");
    const bool rg_on = rge && (rge[0] == '1' || rge[0] == 'f'), rg_force = rge && rge[0] == 'f';
#endif
    const bool rg_tables = s.dev.lds_bytes <= 16 * 1024;
    uint32_t rg_blocks = 0;
    if (rg_on) {
        int per_cu = 0;
        const size_t rl = (rg_tables ? (s.dev.lds_bytes + 15) / 16 * 16 : 0) + rg_state_bytes(L.count) + rg_extra_bytes();
        const void *kf = rg_tables ? reinterpret_cast<const void *>(&check_kernel_rg<false, true>)
                                   : reinterpret_cast<const void *>(&check_kernel_rg<false, false>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, RG, rl) != hipSuccess || per_cu <= 0) per_cu = 1;
        per_cu = std::min(per_cu, KETO_RG_MAX_BLOCKS_PER_CU);
        rg_blocks = (uint32_t)per_cu * cus;
    }
    const bool rg = rg_on && (rg_force || nl >= 4ull * rg_blocks * RG);
    if (rg) rg_blocks = (uint32_t)std::min<uint64_t>(rg_blocks, (nl + RG - 1) / RG);
    for (int tier = 0; tier < 3; tier++) {
        CheckParams P{};
        P.s = s.dev;
        P.start = st.resolved;
        P.qlist = tier == 0 ? list : lists[tier - 1];
        P.qlist_count = tier == 0 ? list_count : &sc.ctrl[3 + tier - 1];
        P.n = (uint32_t)L.n;
        P.out_allowed = L.out_allowed;
        P.out_err = L.out_err;
        P.next = &sc.ctrl[tier];
        P.ovf_list = tier < 2 ? lists[tier] : nullptr;
        P.ovf_count = tier < 2 ? &sc.ctrl[3 + tier] : nullptr;
        P.vis = sc.vis[tier];
        P.stack = sc.stack[tier];
        P.epochs = sc.epochs[tier];
        P.vcap = t[tier].vcap;
        P.scap = t[tier].scap;
        P.max_depth = L.max_depth;
        P.max_width = L.max_width;
        P.counters = st.counters + 8 * tier;
        P.last_tier = tier == 2;
        P.err_detail = L.err_detail;
        uint32_t lanes = t[tier].lanes;
        if (tier == 0) {  // persistent grid: the resident blocks (occupancy API), capped by the batch
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&check_kernel<false, true>),
                                                             BLOCK, lds) != hipSuccess || per_cu <= 0)
                per_cu = 4;
            per_cu = std::min(per_cu, KETO_T0_BLOCKS_PER_CU);
            lanes = std::min<uint32_t>(lanes, (uint32_t)per_cu * cus * BLOCK);
            // A batch smaller than the resident grid is spread over more waves with fewer live
            // lanes each: a wave-step then runs fewer distinct interpreter states, which is what
            // sets the step time (and so a small batch's latency).
            const uint64_t waves = lanes / 64;
            P.live_lanes = (uint32_t)std::min<uint64_t>(64, (nl + waves - 1) / waves);
#ifndef KETO_DFS_OLD
            // queries routed by an asynchronous frontier pass: their number is on the device and is
            // few (C2: ~5 per 2^20, C4: 0), so each gets a wave of its own, as a synchronous pass's
            // few routed queries do -- in one shared wave their divergent steps serialise (C2: up
            // to 0.7 ms per batch instead of 0.15)
            if (count_on_device) P.live_lanes = 1;
#endif
            const uint64_t need = (nl + P.live_lanes - 1) / P.live_lanes * 64;
            lanes = (uint32_t)std::min<uint64_t>(lanes, (need + BLOCK - 1) / BLOCK * BLOCK);
        } else {
            P.live_lanes = 64;
        }
        const uint32_t bs = std::min<uint32_t>(BLOCK, lanes);  // every launched lane owns scratch
        dim3 grid(lanes / bs), block(bs);
        if (tier == 0 && timed) st.mark_begin();
        if (tier == 0 && rg) {  // the block-regrouped interpreter: resident blocks of RG slots
            const size_t rl = (rg_tables ? (s.dev.lds_bytes + 15) / 16 * 16 : 0) + rg_state_bytes(L.count) + rg_extra_bytes();
            dim3 g(rg_blocks), b(RG);
            if (rg_tables) {
                if (L.count) hipLaunchKernelGGL((check_kernel_rg<true, true>), g, b, rl, st.stream, P);
                else hipLaunchKernelGGL((check_kernel_rg<false, true>), g, b, rl, st.stream, P);
            } else {
                if (L.count) hipLaunchKernelGGL((check_kernel_rg<true, false>), g, b, rl, st.stream, P);
                else hipLaunchKernelGGL((check_kernel_rg<false, false>), g, b, rl, st.stream, P);
            }
        } else if (lds_tables) {
            if (L.count) hipLaunchKernelGGL((check_kernel<true, true>), grid, block, lds, st.stream, P);
            else hipLaunchKernelGGL((check_kernel<false, true>), grid, block, lds, st.stream, P);
        } else {
            if (L.count) hipLaunchKernelGGL((check_kernel<true, false>), grid, block, 0, st.stream, P);
            else hipLaunchKernelGGL((check_kernel<false, false>), grid, block, 0, st.stream, P);
        }
        KETO_HIP(hipGetLastError());
        if (tier == 0 && timed) st.mark_end();
    }
}

// Check over a resolved batch: the frontier engine (frontier.hip) answers every query whose
// result cannot depend on visited pruning and routes the rest here; KETO_FRONTIER=0 (A/B) and
// work-counting launches run the DFS interpreter on the whole batch.  The frontier engine's timed
// region is the whole device path of the batch, request resolution (A1) included.
void run_check(const Snapshot &s, Stream &st, const CheckLaunch &L) {
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    const char *fe = getenv("KETO_FRONTIER");
    const bool frontier = !L.count && !(fe && fe[0] == '0');
    if (!frontier) {
        run_resolve(s, st, L.queries, L.q16, L.n, L.max_depth);
        run_dfs(s, st, L, nullptr, nullptr, L.n, true);
        return;
    }
    // Two engines evaluate the same goals (frontier_goal.inc): the generation engine (frontier.hip,
    // a launch per generation over the whole batch) for large batches -- C4 3.7 vs 4.6 ms per 2^20
    // batch -- and the block engine (frontier_block.hip, one launch, a workgroup per chunk of
    // queries) for batches of up to KETO_FR_BLOCK_MAX queries, whose ~32 launches per batch would
    // otherwise set their latency (serving, small batches).  KETO_FR_ENGINE=gen /
    // block forces one.
    static const uint64_t block_max = [] {
        const char *e = getenv("KETO_FR_BLOCK_MAX");
        return e ? (uint64_t)strtoull(e, nullptr, 10) : (uint64_t)1 << 16;
    }();
    const char *ee = getenv("KETO_FR_ENGINE");
    const bool gen = ee ? ee[0] != 'b' : L.n > block_max;
    st.mark_begin();
    run_resolve(s, st, L.queries, L.q16, L.n, L.max_depth, false);
    for (uint64_t off = 0; off < L.n; off += FR_MAX_BATCH) {
        CheckLaunch Lp = L;
        Lp.n = std::min<uint64_t>(FR_MAX_BATCH, L.n - off);
        const uint32_t routed = gen ? run_frontier(s, st, Lp, off) : run_frontier_block(s, st, Lp, off);
        const uint32_t *fl = gen ? st.frontier.fb_list : st.frontier_block.fb_list;
        const uint32_t *fc = gen ? st.frontier.fb_count : st.frontier_block.fb_count;
        // asynchronous: the interpreter is sized for the whole pass and reads the routed count on
        // the device (its lanes find an empty list and leave)
        if (routed) run_dfs(s, st, L, fl, fc, routed == FR_ROUTED_ON_DEVICE ? Lp.n : routed, false, routed == FR_ROUTED_ON_DEVICE);
    }
    st.mark_end();
}

}  // namespace keto
