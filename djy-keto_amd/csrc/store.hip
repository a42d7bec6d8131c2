// Incremental snapshots: a device-resident tuple store that takes
// TransactRelationTuples deltas and cuts versioned snapshots.
//
// Reference semantics, persistence/sql/relationtuples.go:
//   TransactRelationTuples(ins, del) (:277-287) = WriteRelationTuples(ins) then
//   DeleteRelationTuples(del), in one transaction.
//   - Every insert is a new row with a fresh UUIDv4 shard_id (:104-126, no content
//     uniqueness: the same tuple may be stored twice).
//   - A delete removes every row whose (namespace, object, relation, subject) matches,
//     including rows inserted by the same transaction (:168-189).  A subject id matches
//     on subject_id alone, a subject set on its three fields (whereSubject, :128-150).
// The shim supplies the inserted rows' shard_ids (it writes the same rows to SQL).
//
// On the device: inserts are appended; deletes go through an open-addressing hash of the
// delete keys and one pass over the store that flags matching rows.  Survivors are then
// compacted in place: the deleted slots below the new length are filled with the live rows
// above it.  Row order does not matter, because the snapshot builder orders every row by
// shard_id.  A snapshot of the current content is stamped with the store's version: the
// snaptoken the reference leaves unimplemented (check/handler.go:327-330).  It is either one
// device build (keto_snapshot_build_device, ~2 s at 1B tuples) or a patch of an earlier
// snapshot of this store (patch.hip): the store keeps every transaction's rows in a change log
// (bounded), and the rows they name are the only ones a patch rebuilds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <memory>
#include <vector>

#include "engine.hpp"

namespace keto {
namespace {

constexpr uint32_t BLK = 256;
inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, (n + BLK - 1) / BLK)); }
__device__ __forceinline__ uint64_t gid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// the matched content of a row: subject sets compare ns/obj/rel, subject ids only the id
struct Key {
    uint32_t ns, obj, rel, kind, s_obj, s_ns, s_rel;
};
__device__ __forceinline__ Key key_of(const keto_tuple &t) {
    const bool set = t.subj_kind == 1;
    return Key{t.ns, t.obj, t.rel, set ? 1u : 0u, t.s_obj, set ? t.s_ns : 0u, set ? t.s_rel : 0u};
}
__device__ __forceinline__ bool same(const Key &a, const Key &b) {
    return a.ns == b.ns && a.obj == b.obj && a.rel == b.rel && a.kind == b.kind && a.s_obj == b.s_obj &&
           a.s_ns == b.s_ns && a.s_rel == b.s_rel;
}
__device__ __forceinline__ uint64_t key_hash(const Key &k) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    const uint32_t w[7] = {k.ns, k.obj, k.rel, k.kind, k.s_obj, k.s_ns, k.s_rel};
    for (int i = 0; i < 7; i++) {
        h ^= w[i];
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
    }
    return h;
}

// slot = index of a delete key + 1 (0 = empty); duplicates of one key may share the table
__global__ __launch_bounds__(BLK) void k_del_insert(const keto_tuple *del, uint64_t n, uint32_t *slots, uint64_t mask) {
    const uint64_t i = gid();
    if (i >= n) return;
    uint64_t h = key_hash(key_of(del[i])) & mask;
    for (;;) {
        if (atomicCAS(&slots[h], 0u, (uint32_t)(i + 1)) == 0u) return;
        h = (h + 1) & mask;
    }
}

__global__ __launch_bounds__(BLK) void k_mark(const keto_tuple *t, uint64_t n, const keto_tuple *del,
                                              const uint32_t *slots, uint64_t mask, uint8_t *dead,
                                              unsigned long long *n_dead) {
    const uint64_t i = gid();
    if (i >= n) return;
    const Key k = key_of(t[i]);
    uint64_t h = key_hash(k) & mask;
    bool hit = false;
    for (;;) {
        const uint32_t s = slots[h];
        if (s == 0u) break;
        if (same(key_of(del[s - 1]), k)) {
            hit = true;
            break;
        }
        h = (h + 1) & mask;
    }
    dead[i] = hit ? 1 : 0;
    if (hit) atomicAdd(n_dead, 1ull);
}

// holes: dead rows below the new length; movers: live rows at or above it (equal counts)
__global__ __launch_bounds__(BLK) void k_holes_movers(const uint8_t *dead, uint64_t n, uint64_t keep, uint64_t *holes,
                                                      uint64_t *movers, unsigned long long *cnt) {
    const uint64_t i = gid();
    if (i >= n) return;
    if (i < keep && dead[i]) holes[atomicAdd(&cnt[0], 1ull)] = i;
    if (i >= keep && !dead[i]) movers[atomicAdd(&cnt[1], 1ull)] = i;
}

__global__ __launch_bounds__(BLK) void k_move(keto_tuple *t, const uint64_t *holes, const uint64_t *movers, uint64_t m) {
    const uint64_t i = gid();
    if (i >= m) return;
    t[holes[i]] = t[movers[i]];
}

}  // namespace

struct TupleStore {
    int device = 0;
    build::DevBuf buf;  // capacity in rows = buf.bytes / sizeof(keto_tuple)
    uint64_t n = 0, version = 0;
    uint64_t id = 0;  // stamped on its snapshots: a patch only takes a base cut from this store
    // change log: the rows of the last transactions (inserts then deletes), oldest first
    struct Change {
        uint64_t version, n_ins, n_del;
        build::DevBuf rows;
    };
    std::deque<Change> log;
    uint64_t log_rows = 0;
    static constexpr uint64_t LOG_MAX_ROWS = 1ull << 22;
    keto_tuple *rows() const { return static_cast<keto_tuple *>(buf.p); }
    uint64_t cap() const { return buf.bytes / sizeof(keto_tuple); }
    void reserve(uint64_t need) {
        if (need <= cap()) return;
        build::DevBuf nb(std::max<uint64_t>(need, cap() + cap() / 4) * sizeof(keto_tuple));
        if (n) KETO_HIP(hipMemcpy(nb.p, buf.p, n * sizeof(keto_tuple), hipMemcpyDeviceToDevice));
        buf = std::move(nb);
    }
};

TupleStore *store_create(int device, const keto_tuple *tuples, uint64_t n, bool device_ptrs) {
    KETO_HIP(hipSetDevice(device));
    static std::atomic<uint64_t> next_id{1};
    auto st = std::make_unique<TupleStore>();
    st->device = device;
    st->id = next_id++;
    st->reserve(std::max<uint64_t>(n + n / 16 + (1u << 16), 64));  // (room for transactions: no regrowth copy)
    if (n)
        KETO_HIP(hipMemcpy(st->rows(), tuples, n * sizeof(keto_tuple),
                           device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    st->n = n;
    return st.release();
}

void store_transact(TupleStore &st, const keto_tuple *ins, uint64_t n_ins, const keto_tuple *del, uint64_t n_del,
                    bool device_ptrs) {
    KETO_HIP(hipSetDevice(st.device));
    const hipMemcpyKind kind = device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    // the change log entry of this version, logged only once the transaction has been applied
    // (next to version++): a transaction that throws part-way leaves neither an entry nor a new
    // version.  (A transaction larger than the log holds none: a snapshot across it is a full build.)
    TupleStore::Change c{st.version + 1, n_ins, n_del, build::DevBuf(sizeof(keto_tuple) * std::max<uint64_t>(1, n_ins + n_del))};
    if (n_ins) KETO_HIP(hipMemcpy(c.rows.p, ins, n_ins * sizeof(keto_tuple), kind));
    if (n_del) KETO_HIP(hipMemcpy(static_cast<keto_tuple *>(c.rows.p) + n_ins, del, n_del * sizeof(keto_tuple), kind));
    const uint64_t n_before = st.n;
    if (n_ins) {  // WriteRelationTuples: appended rows, fresh shard_ids from the caller
        st.reserve(st.n + n_ins);
        KETO_HIP(hipMemcpy(st.rows() + st.n, ins, n_ins * sizeof(keto_tuple), kind));
    }
    // (the appended rows count only once the deletes below went through: st.n stays n_before
    // until the end, so a throw leaves the store's content as it was)
    const uint64_t n_all = n_before + n_ins;
    uint64_t n_after = n_all;
    if (n_del && n_all) {  // DeleteRelationTuples over everything, the new rows included
        build::DevBuf d(n_del * sizeof(keto_tuple));
        KETO_HIP(hipMemcpy(d.p, del, n_del * sizeof(keto_tuple), kind));
        uint64_t size = 64;
        while (size < 2 * n_del) size <<= 1;
        build::DevBuf slots(size * 4), dead(n_all), cnt(3 * sizeof(unsigned long long));
        KETO_HIP(hipMemset(slots.p, 0, size * 4));
        KETO_HIP(hipMemset(cnt.p, 0, 3 * sizeof(unsigned long long)));
        auto *cn = static_cast<unsigned long long *>(cnt.p);
        hipLaunchKernelGGL(k_del_insert, grid_for(n_del), dim3(BLK), 0, 0, static_cast<const keto_tuple *>(d.p), n_del,
                           slots.u32(), size - 1);
        KETO_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_mark, grid_for(n_all), dim3(BLK), 0, 0, st.rows(), n_all,
                           static_cast<const keto_tuple *>(d.p), slots.u32(), size - 1,
                           static_cast<uint8_t *>(dead.p), cn + 2);
        KETO_HIP(hipGetLastError());
        unsigned long long n_dead = 0;
        KETO_HIP(hipMemcpy(&n_dead, cn + 2, sizeof(n_dead), hipMemcpyDeviceToHost));
        if (n_dead) {
            const uint64_t keep = n_all - n_dead;
            build::DevBuf holes(n_dead * 8), movers(n_dead * 8);
            hipLaunchKernelGGL(k_holes_movers, grid_for(n_all), dim3(BLK), 0, 0, static_cast<const uint8_t *>(dead.p),
                               n_all, keep, static_cast<uint64_t *>(holes.p), static_cast<uint64_t *>(movers.p), cn);
            KETO_HIP(hipGetLastError());
            unsigned long long m[2] = {0, 0};
            KETO_HIP(hipMemcpy(m, cn, sizeof(m), hipMemcpyDeviceToHost));
            if (m[0] != m[1]) throw Error(KETO_E_DEVICE, "compaction lists disagree");
            hipLaunchKernelGGL(k_move, grid_for(m[0]), dim3(BLK), 0, 0, st.rows(),
                               static_cast<const uint64_t *>(holes.p), static_cast<const uint64_t *>(movers.p), m[0]);
            KETO_HIP(hipGetLastError());
            n_after = keep;
        }
    }
    KETO_HIP(hipDeviceSynchronize());
    // applied: the new content, its version and its log entry together
    st.n = n_after;
    st.version++;
    st.log_rows += n_ins + n_del;
    st.log.push_back(std::move(c));
    while (!st.log.empty() && st.log_rows > TupleStore::LOG_MAX_ROWS) {
        st.log_rows -= st.log.front().n_ins + st.log.front().n_del;
        st.log.pop_front();
    }
}

static bool log_since(const TupleStore &st, uint64_t version, build::DevBuf &rows, std::vector<uint8_t> &is_ins);

bool store_snapshot_advance(const TupleStore &st, Snapshot &snap) {
    // the same compiled configuration is implied: snap was cut from this store and keeps its tables
    if (snap.store_id != st.id || snap.device != st.device || snap.info.version > st.version) return false;
    if (snap.info.version == st.version) return true;
    build::DevBuf rows;
    std::vector<uint8_t> is_ins;
    if (!log_since(st, snap.info.version, rows, is_ins)) return false;
    if (!advance_snapshot(snap, static_cast<const keto_tuple *>(rows.p), is_ins.data(), is_ins.size(), st.n)) return false;
    snap.info.version = st.version;
    return true;
}

void store_free(TupleStore *st) { delete st; }

void store_info(const TupleStore &st, uint64_t *n, uint64_t *version) {
    if (n) *n = st.n;
    if (version) *version = st.version;
}

// the arrays a patch of snapshot s will allocate, reserved in the device pool now (a fresh
// multi-GB allocation is cleared by the driver at first use: seconds at 1B tuples), with room
// for the row arrays to grow.  Only at a full cut: in a chain of patches each released version
// hands its arrays to the next patch.
static void reserve_next_patch(const Snapshot &s) {
    const uint64_t N = s.dev.n_nodes, M = (uint64_t)s.dev.n_uuids + N, n = s.info.n_tuples, ne = s.info.n_set_edges;
    auto r = [](uint64_t b) { return (size_t)((b + 31) / 16 * 16); };
    auto grow = [&](uint64_t b) { return r(b + b / 16 + (1u << 20)); };
    pool_reserve(s.device, {r(16 * N), r(4 * (N + 1)), grow(4 * n), r(4 * (M + 1)), grow(4 * n), grow(4 * ne + 16),
                            r(16 * ((uint64_t)s.dev.probe_mask + 1))});
}

Snapshot *store_snapshot(const TupleStore &st, const keto_snapshot_config *cfg) {
    if (!cfg || cfg->device != st.device) throw Error(KETO_E_INVALID, "config names another device");
    // room for what later transactions create, so their patches need no full build: an id space
    // past the caller's (ids not yet written are unknown objects and subjects, as before) and
    // spare entities in every namespace (patch.hip places new objects on them)
    BuildOpts o;
    o.uuid_capacity = (uint32_t)std::min<uint64_t>(0x7FFFFFFFull, (uint64_t)cfg->n_uuids + cfg->n_uuids / 16 + 65536);
    o.spares = true;
    o.room = true;  // (keto_store_snapshot_advance)
    Snapshot *s = build_snapshot(cfg, st.rows(), st.n, true, true, &o);
    s->info.version = st.version;
    s->store_id = st.id;
    reserve_next_patch(*s);
    return s;
}

// the rows of every transaction after `version`, in order (each one's inserts, then its deletes);
// false when the log no longer holds them all, each once
static bool log_since(const TupleStore &st, uint64_t version, build::DevBuf &rows, std::vector<uint8_t> &is_ins) {
    uint64_t want = version + 1, n_rows = 0;
    bool covered = true;
    for (const auto &c : st.log)
        if (c.version > version) {
            if (c.version != want) covered = false;
            want++;
            n_rows += c.n_ins + c.n_del;
        }
    if (!covered || want != st.version + 1) return false;
    KETO_HIP(hipSetDevice(st.device));
    rows = build::DevBuf(sizeof(keto_tuple) * std::max<uint64_t>(1, n_rows));
    is_ins.assign(n_rows, 0);
    uint64_t at = 0;
    for (const auto &c : st.log) {
        if (c.version <= version) continue;
        const uint64_t k = c.n_ins + c.n_del;
        if (k) KETO_HIP(hipMemcpy(static_cast<keto_tuple *>(rows.p) + at, c.rows.p, k * sizeof(keto_tuple), hipMemcpyDeviceToDevice));
        std::fill(is_ins.begin() + at, is_ins.begin() + at + c.n_ins, 1);
        at += k;
    }
    return true;
}

Snapshot *store_snapshot_patch(const TupleStore &st, const Snapshot &base, const keto_snapshot_config *cfg, bool *patched) {
    if (!cfg || cfg->device != st.device) throw Error(KETO_E_INVALID, "config names another device");
    // a patch reuses base's compiled namespaces, name tables and id space: only for the same
    // configuration (a namespace reload, renamed relations or a larger uuid space build in full)
    if (base.store_id == st.id && base.device == st.device && base.info.version <= st.version &&
        base.cfg_hash == config_hash(cfg) && cfg->n_uuids <= base.n_uuids) {
        build::DevBuf rows;
        std::vector<uint8_t> is_ins;
        if (log_since(st, base.info.version, rows, is_ins)) {
            Snapshot *s = patch_snapshot(base, st.rows(), st.n, static_cast<const keto_tuple *>(rows.p), is_ins.data(), is_ins.size());
            if (s) {
                s->info.version = st.version;
                s->store_id = st.id;
                if (patched) *patched = true;  // (the next patch takes this one's base's arrays once it is released)
                return s;
            }
        }
    }
    if (patched) *patched = false;
    return store_snapshot(st, cfg);
}

}  // namespace keto
