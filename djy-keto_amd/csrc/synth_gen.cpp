// Seeded synthetic Drive-style workloads (BASELINE configs 3 and 4):
// bench/test infrastructure, built into its own libketo_synth.so -- never part of the engine.
//
// File/Folder forest: `roots` trees of fanout F and depth D (levels 0..D-1 are folders, level D
// files), one `parents` tuple per non-root node; A ACL tuples per node (50% viewers, 20% editors,
// 20% owners, 10% banned; 30% of the non-banned ones name Group#members, the rest a user);
// G groups x M members (mostly users, ~1 nested group each, acyclic: subgroup id > group id).
// C3 = 1 root, 1M groups, 10M users (~105M tuples); C4 = C3 x 10 (10 roots, 10M groups,
// 100M users: ~1.05B tuples).
//
// Every value is a pure function of (seed, stream, index) through splitmix64, so the arrays
// fill in parallel and every rank of a multi-GPU run regenerates the identical replica.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/keto_mi355x.h"

namespace {

constexpr uint32_t NS_USER = 0, NS_GROUP = 1, NS_FOLDER = 2, NS_FILE = 3;
// relation ids: the order of synth.DRIVE_RELATIONS
constexpr uint32_t R_PARENTS = 0, R_VIEWERS = 1, R_EDITORS = 2, R_OWNERS = 3, R_BANNED = 4, R_VIEW = 5,
                   R_EDIT = 6, R_MEMBERS = 7, R_EMPTY = 8;

inline uint64_t sm64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
inline uint64_t hsh(uint64_t seed, uint64_t stream, uint64_t i) { return sm64(sm64(seed ^ (stream << 48)) ^ i); }
inline double u01(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

template <class F>
void parallel_chunks(uint64_t n, int threads, F fn) {
    threads = std::max(1, std::min(threads, 64));
    if (n < (1u << 16) || threads == 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([=] { fn(n * t / threads, n * (t + 1) / threads); });
    for (auto &x : th) x.join();
}

}  // namespace

extern "C" {

typedef struct ks_drive_params {
    uint32_t roots, depth, fanout, acl_per_node;
    uint32_t n_groups, members_per_group, n_users, pad;
    uint64_t seed;
} ks_drive_params;

typedef struct ks_drive_layout {
    uint64_t nodes_per_root, folders_per_root, n_nodes;
    uint64_t n_parent_tuples, n_acl_tuples, n_member_tuples, n_tuples;
    uint64_t gbase, ubase, n_uuids;
} ks_drive_layout;

int ks_drive_layout_get(const ks_drive_params *p, ks_drive_layout *L) {
    if (!p || !L || p->fanout < 2 || p->roots == 0 || p->n_groups == 0 || p->n_users == 0) return -1;
    uint64_t per = 0, lvl = 1, folders = 0;
    for (uint32_t k = 0; k <= p->depth; k++) {
        per += lvl;
        if (k < p->depth) folders += lvl;
        lvl *= p->fanout;
    }
    L->nodes_per_root = per;
    L->folders_per_root = folders;
    L->n_nodes = per * p->roots;
    L->n_parent_tuples = (per - 1) * p->roots;
    L->n_acl_tuples = L->n_nodes * p->acl_per_node;
    L->n_member_tuples = (uint64_t)p->n_groups * p->members_per_group;
    L->n_tuples = L->n_parent_tuples + L->n_acl_tuples + L->n_member_tuples;
    L->gbase = L->n_nodes;
    L->ubase = L->n_nodes + p->n_groups;
    L->n_uuids = L->ubase + p->n_users;
    return L->n_uuids < 0x80000000ull ? 0 : -2;
}

static inline uint32_t node_ns(const ks_drive_layout &L, uint64_t node) {
    return node % L.nodes_per_root < L.folders_per_root ? NS_FOLDER : NS_FILE;
}

// ACL tuple j: (relation, is-group, subject uuid)
static inline void acl_of(const ks_drive_params &p, const ks_drive_layout &L, uint64_t j, uint32_t &rel, bool &grp,
                          uint32_t &subj) {
    const double r = u01(hsh(p.seed, 1, j));
    rel = r < 0.5 ? R_VIEWERS : (r < 0.7 ? R_EDITORS : (r < 0.9 ? R_OWNERS : R_BANNED));
    grp = rel != R_BANNED && u01(hsh(p.seed, 2, j)) < 0.3;
    subj = grp ? (uint32_t)(L.gbase + hsh(p.seed, 3, j) % p.n_groups) : (uint32_t)(L.ubase + hsh(p.seed, 4, j) % p.n_users);
}

static inline void shard(const ks_drive_params &p, uint64_t i, uint8_t *b) {
    uint64_t a = hsh(p.seed, 8, i), c = hsh(p.seed, 9, i);
    for (int k = 0; k < 8; k++) {
        b[k] = (uint8_t)(a >> (8 * k));
        b[8 + k] = (uint8_t)(c >> (8 * k));
    }
    b[6] = (b[6] & 0x0F) | 0x40;  // UUIDv4 version
    b[8] = (b[8] & 0x3F) | 0x80;  // RFC 4122 variant
}

static inline keto_tuple drive_tuple(const ks_drive_params &p, const ks_drive_layout &L, uint64_t i) {
    keto_tuple t{};
    if (i < L.n_parent_tuples) {  // node#parents@Folder:parent#""
        const uint64_t r = i / (L.nodes_per_root - 1), c = 1 + i % (L.nodes_per_root - 1);
        const uint64_t node = r * L.nodes_per_root + c, par = r * L.nodes_per_root + (c - 1) / p.fanout;
        t.ns = node_ns(L, node);
        t.obj = (uint32_t)node;
        t.rel = R_PARENTS;
        t.subj_kind = 1;
        t.s_obj = (uint32_t)par;
        t.s_ns = NS_FOLDER;
        t.s_rel = R_EMPTY;
    } else if (i < L.n_parent_tuples + L.n_acl_tuples) {
        const uint64_t j = i - L.n_parent_tuples, node = j / p.acl_per_node;
        uint32_t rel, subj;
        bool grp;
        acl_of(p, L, j, rel, grp, subj);
        t.ns = node_ns(L, node);
        t.obj = (uint32_t)node;
        t.rel = rel;
        t.subj_kind = grp ? 1 : 0;
        t.s_obj = subj;
        t.s_ns = grp ? NS_GROUP : 0;
        t.s_rel = grp ? R_MEMBERS : 0;
    } else {  // Group:g#members@(user | Group:sub#members), sub > g
        const uint64_t k = i - L.n_parent_tuples - L.n_acl_tuples, g = k / p.members_per_group;
        const bool nested = g + 1 < p.n_groups && u01(hsh(p.seed, 5, k)) < 1.0 / p.members_per_group;
        t.ns = NS_GROUP;
        t.obj = (uint32_t)(L.gbase + g);
        t.rel = R_MEMBERS;
        if (nested) {
            const uint64_t span = p.n_groups - g - 1;
            const uint64_t sub = g + 1 + std::min<uint64_t>(span - 1, (uint64_t)(u01(hsh(p.seed, 6, k)) * span));
            t.subj_kind = 1;
            t.s_obj = (uint32_t)(L.gbase + sub);
            t.s_ns = NS_GROUP;
            t.s_rel = R_MEMBERS;
        } else {
            t.s_obj = (uint32_t)(L.ubase + hsh(p.seed, 7, k) % p.n_users);
        }
    }
    shard(p, i, t.shard_id);
    return t;
}

int ks_drive_tuples(const ks_drive_params *pp, keto_tuple *out, uint64_t n, int threads) {
    ks_drive_layout L;
    if (ks_drive_layout_get(pp, &L) != 0 || n != L.n_tuples || !out) return -1;
    const ks_drive_params p = *pp;
    parallel_chunks(n, threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) out[i] = drive_tuple(p, L, i);
    });
    return 0;
}

// The tuples whose object belongs to partition `part` of `nparts` (keto_object_owner): what one
// rank of a partitioned (config 5) job loads.  out == NULL only counts.  The walk is over
// objects -- a node's parents + ACL tuples, a group's member tuples -- so the owner test runs
// once per object and only the partition's own tuples are generated (every rank of an 8-way
// job scans the object space, not the 4.2B-tuple index space); two passes (count per chunk,
// then fill at exact offsets), so no partition ever needs the whole graph in host memory.
int ks_drive_tuples_part_placed(const ks_drive_params *pp, uint32_t nparts, uint32_t part, const keto_placement *pl,
                                keto_tuple *out, uint64_t cap, int threads, uint64_t *count);
int ks_drive_tuples_part(const ks_drive_params *pp, uint32_t nparts, uint32_t part, keto_tuple *out, uint64_t cap,
                         int threads, uint64_t *count) {
    return ks_drive_tuples_part_placed(pp, nparts, part, nullptr, out, cap, threads, count);
}
// the same under a placement (keto_object_owner_placed; null: keto_object_owner)
int ks_drive_tuples_part_placed(const ks_drive_params *pp, uint32_t nparts, uint32_t part, const keto_placement *pl,
                                keto_tuple *out, uint64_t cap, int threads, uint64_t *count) {
    ks_drive_layout L;
    if (ks_drive_layout_get(pp, &L) != 0 || nparts == 0 || part >= nparts || !count) return -1;
    const ks_drive_params p = *pp;
    const int T = std::max(1, std::min(threads, 64));
    const uint64_t n_obj = L.n_nodes + p.n_groups;  // objects: nodes, then groups
    std::vector<uint64_t> cnt(T + 1, 0);
    auto run = [&](bool fill) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                const uint64_t b = n_obj * t / T, e = n_obj * (t + 1) / T;
                uint64_t c = 0, o = fill ? cnt[t] : 0;
                auto emit = [&](uint64_t i) {
                    if (fill) out[o++] = drive_tuple(p, L, i);
                    c++;
                };
                for (uint64_t x = b; x < e; x++) {
                    if (x < L.n_nodes) {
                        const uint32_t o = keto_object_owner_placed(pl, node_ns(L, x), (uint32_t)x, nparts);
                        if (o != part && o != KETO_OWNER_ALL) continue;
                        const uint64_t r = x / L.nodes_per_root, cc = x % L.nodes_per_root;
                        if (cc) emit(r * (L.nodes_per_root - 1) + cc - 1);
                        for (uint64_t a = 0; a < p.acl_per_node; a++) emit(L.n_parent_tuples + x * p.acl_per_node + a);
                    } else {
                        const uint64_t g = x - L.n_nodes;
                        const uint32_t o = keto_object_owner_placed(pl, NS_GROUP, (uint32_t)(L.gbase + g), nparts);
                        if (o != part && o != KETO_OWNER_ALL) continue;
                        for (uint64_t m = 0; m < p.members_per_group; m++)
                            emit(L.n_parent_tuples + L.n_acl_tuples + g * p.members_per_group + m);
                    }
                }
                if (!fill) cnt[t + 1] = c;
            });
        for (auto &x : th) x.join();
    };
    run(false);
    for (int t = 0; t < T; t++) cnt[t + 1] += cnt[t];
    *count = cnt[T];
    if (!out) return 0;
    if (cap < cnt[T]) return -2;
    run(true);
    return 0;
}

// Every tuple of the given objects (keys = ns << 32 | obj), straight from the generator's index
// space -- a node's parents tuple and its ACL tuples, a group's member tuples; users own none --
// so a test can collect the closure of a batch on a multi-billion-tuple graph without holding
// it.  out == NULL only counts; objects are emitted in key order, tuples in generation order.
int ks_drive_object_tuples(const ks_drive_params *pp, const uint64_t *keys, uint64_t n, keto_tuple *out, uint64_t cap,
                           uint64_t *count) {
    ks_drive_layout L;
    if (ks_drive_layout_get(pp, &L) != 0 || !count || (n && !keys)) return -1;
    const ks_drive_params p = *pp;
    uint64_t c = 0;
    auto emit = [&](uint64_t i) {
        if (out && c < cap) out[c] = drive_tuple(p, L, i);
        c++;
    };
    for (uint64_t k = 0; k < n; k++) {
        const uint32_t ns = (uint32_t)(keys[k] >> 32);
        const uint64_t obj = (uint32_t)keys[k];
        if ((ns == NS_FOLDER || ns == NS_FILE) && obj < L.n_nodes && node_ns(L, obj) == ns) {
            const uint64_t r = obj / L.nodes_per_root, cc = obj % L.nodes_per_root;
            if (cc) emit(r * (L.nodes_per_root - 1) + cc - 1);
            for (uint64_t a = 0; a < p.acl_per_node; a++) emit(L.n_parent_tuples + obj * p.acl_per_node + a);
        } else if (ns == NS_GROUP && obj >= L.gbase && obj < L.gbase + p.n_groups) {
            const uint64_t g = obj - L.gbase;
            for (uint64_t m = 0; m < p.members_per_group; m++)
                emit(L.n_parent_tuples + L.n_acl_tuples + g * p.members_per_group + m);
        }
    }
    *count = c;
    return out && c > cap ? -2 : 0;
}

// view (80%) / edit checks: half name a user taken from a random user ACL tuple of the queried
// node (likely positives, unless banned or truncated), half a uniform node and user.
int ks_drive_queries(const ks_drive_params *pp, uint64_t qseed, keto_query *out, uint64_t n, int threads) {
    ks_drive_layout L;
    if (ks_drive_layout_get(pp, &L) != 0 || !out) return -1;
    const ks_drive_params p = *pp;
    parallel_chunks(n, threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            keto_query q{};
            uint64_t node;
            uint32_t user;
            if (u01(hsh(qseed, 1, i)) < 0.5) {
                for (uint64_t t = 0;; t++) {
                    const uint64_t j = hsh(qseed, 2, i * 64 + t) % L.n_acl_tuples;
                    uint32_t rel, subj;
                    bool grp;
                    acl_of(p, L, j, rel, grp, subj);
                    if ((rel == R_VIEWERS || rel == R_EDITORS || rel == R_OWNERS) && !grp) {
                        node = j / p.acl_per_node;
                        user = subj;
                        break;
                    }
                }
            } else {
                node = hsh(qseed, 3, i) % L.n_nodes;
                user = (uint32_t)(L.ubase + hsh(qseed, 4, i) % p.n_users);
            }
            q.ns = node_ns(L, node);
            q.obj = (uint32_t)node;
            q.rel = u01(hsh(qseed, 5, i)) < 0.8 ? R_VIEW : R_EDIT;
            q.subj_kind = 0;
            q.s_obj = user;
            q.max_depth = 0;
            out[i] = q;
        }
    });
    return 0;
}

// Closed-loop serving load (bench infrastructure): `clients` native threads each send `req`-query
// requests back to back through `check` (keto_dispatcher_check, passed in by the caller) for
// `seconds`, the way goroutines of the Go shim would call it through cgo.  Per-request latency
// percentiles over all threads.
typedef int (*ks_check_fn)(void *dispatcher, const keto_query *queries, uint64_t n, uint8_t *out_allowed,
                           int32_t *out_err);
typedef struct ks_load_result {
    uint64_t requests, checks;
    double seconds, p50_ms, p99_ms, max_ms;
    int32_t rc;  // first non-zero return code of any request, else 0
} ks_load_result;

int ks_closed_loop(ks_check_fn check, void *dispatcher, const keto_query *queries, uint64_t nq, uint32_t clients,
                   uint32_t req, double seconds, ks_load_result *out) {
    if (!check || !dispatcher || !queries || !out || clients == 0 || req == 0 || nq < req) return -1;
    using clk = std::chrono::steady_clock;
    const auto stop = clk::now() + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(seconds));
    std::vector<std::vector<float>> lat(clients);
    std::vector<int32_t> rcs(clients, 0);
    const uint64_t span = nq - req + 1;
    const auto t0 = clk::now();
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < clients; t++)
        th.emplace_back([&, t] {
            std::vector<uint8_t> allowed(req);
            std::vector<int32_t> err(req);
            uint64_t i = ((uint64_t)t * 7919u * req) % span;
            while (clk::now() < stop) {
                const auto a = clk::now();
                const int rc = check(dispatcher, queries + i, req, allowed.data(), err.data());
                const auto b = clk::now();
                if (rc != 0) {
                    rcs[t] = rc;
                    return;
                }
                lat[t].push_back(std::chrono::duration<float, std::milli>(b - a).count());
                i = (i + (uint64_t)clients * req) % span;
            }
        });
    for (auto &x : th) x.join();
    const double dt = std::chrono::duration<double>(clk::now() - t0).count();
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    out->rc = 0;
    for (int32_t r : rcs)
        if (r != 0 && out->rc == 0) out->rc = r;
    out->requests = all.size();
    out->checks = all.size() * (uint64_t)req;
    out->seconds = dt;
    out->p50_ms = out->p99_ms = out->max_ms = 0;
    if (!all.empty()) {
        std::sort(all.begin(), all.end());
        auto pct = [&](double p) { return (double)all[std::min<size_t>(all.size() - 1, (size_t)(p * all.size()))]; };
        out->p50_ms = pct(0.50);
        out->p99_ms = pct(0.99);
        out->max_ms = all.back();
    }
    return 0;
}

}  // extern "C"
