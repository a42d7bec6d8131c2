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
// On the device: inserts are appended; deletes find their rows through the store's content
// index -- open addressing over {32-bit tag of the content hash, row position}, every stored row
// once, the reference's SQL index on the same columns -- so a transaction costs its own rows, not
// the store.  Survivors are then compacted in place: the deleted slots below the new length are
// filled with the live rows above it (the index entries of the moved rows repointed).  Row order
// does not matter, because the snapshot builder orders every row by shard_id.  A snapshot of the current content is stamped with the store's version: the
// snaptoken the reference leaves unimplemented (check/handler.go:327-330).  It is either one
// device build (keto_snapshot_build_device, ~2 s at 1B tuples) or a patch of an earlier
// snapshot of this store (patch.hip): the store keeps every transaction's rows in a change log
// (bounded), and the rows they name are the only ones a patch rebuilds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

// ---- the content index: entry = tag << 32 | position (IX_EMPTY: free, IX_TOMB: a deleted row's) ----
constexpr uint32_t IX_EMPTY = 0xFFFFFFFFu, IX_TOMB = 0xFFFFFFFEu;
struct Ix {
    unsigned long long *slot;
    uint32_t n;  // slots (< 2^32: home = multiply-shift of the hash's low word)
};
__device__ __forceinline__ uint32_t ix_home(const Ix &x, uint64_t h) { return (uint32_t)(((h & 0xFFFFFFFFull) * x.n) >> 32); }
__device__ __forceinline__ uint32_t ix_next(const Ix &x, uint32_t b) { return b + 1 == x.n ? 0u : b + 1; }

__global__ __launch_bounds__(BLK) void k_ix_insert(const keto_tuple *t, uint64_t first, uint64_t n, Ix x) {
    const uint64_t i = gid();
    if (i >= n) return;
    const uint64_t pos = first + i, h = key_hash(key_of(t[pos]));
    const unsigned long long e = (h >> 32) << 32 | pos;
    for (uint32_t b = ix_home(x, h);; b = ix_next(x, b)) {
        unsigned long long cur = x.slot[b];
        while ((uint32_t)cur == IX_EMPTY) {
            const unsigned long long was = atomicCAS(&x.slot[b], cur, e);
            if (was == cur) return;
            cur = was;
        }
    }
}

// every live row matching a delete key: its entry becomes a tombstone (one CAS: a key listed twice
// takes each row once) and its position goes to the dead list
__global__ __launch_bounds__(BLK) void k_ix_delete(const keto_tuple *t, const keto_tuple *del, uint64_t n_del, Ix x, uint32_t *dead,
                                                   uint64_t cap, unsigned long long *n_dead) {
    const uint64_t i = gid();
    if (i >= n_del) return;
    const Key k = key_of(del[i]);
    const uint64_t h = key_hash(k);
    const uint32_t tag = (uint32_t)(h >> 32);
    for (uint32_t b = ix_home(x, h);; b = ix_next(x, b)) {
        const unsigned long long cur = x.slot[b];
        const uint32_t pos = (uint32_t)cur;
        if (pos == IX_EMPTY) return;
        if (pos == IX_TOMB || (uint32_t)(cur >> 32) != tag || !same(key_of(t[pos]), k)) continue;
        if (atomicCAS(&x.slot[b], cur, (unsigned long long)tag << 32 | IX_TOMB) == cur) {
            const unsigned long long at = atomicAdd(n_dead, 1ull);
            if (at < cap) dead[at] = pos;
        }
    }
}

// the live rows above the new length into the deleted slots below it, their entries repointed
__global__ __launch_bounds__(BLK) void k_ix_move(keto_tuple *t, const uint2 *moves, uint64_t m, Ix x) {
    const uint64_t i = gid();
    if (i >= m) return;
    const uint32_t from = moves[i].x, to = moves[i].y;
    const keto_tuple row = t[from];
    t[to] = row;
    const uint64_t h = key_hash(key_of(row));
    const unsigned long long e = (h >> 32) << 32 | from;
    for (uint32_t b = ix_home(x, h);; b = ix_next(x, b)) {
        const unsigned long long cur = x.slot[b];
        if ((uint32_t)cur == IX_EMPTY) return;  // (not reached: every stored row has its entry)
        if (cur == e) {
            x.slot[b] = (h >> 32) << 32 | to;
            return;
        }
    }
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
    // the content index: 3/2 slots per row of capacity, entries and tombstones counted
    build::DevBuf ix;
    uint64_t ix_slots = 0, ix_used = 0;
    bool ix_dirty = false;  // a transaction threw part-way: entries past n may exist (re-index first)
    keto_tuple *rows() const { return static_cast<keto_tuple *>(buf.p); }
    uint64_t cap() const { return buf.bytes / sizeof(keto_tuple); }
    Ix index() const { return Ix{static_cast<unsigned long long *>(ix.p), (uint32_t)ix_slots}; }
    void reserve(uint64_t need) {
        if (need <= cap()) return;
        if (need >= 0xFFFFFFF0ull) throw Error(KETO_E_LIMIT, "a store of 2^32 rows");
        build::DevBuf nb(std::min<uint64_t>(0xFFFFFFF0ull, std::max<uint64_t>(need, cap() + cap() / 4)) * sizeof(keto_tuple));
        if (n) KETO_HIP(hipMemcpy(nb.p, buf.p, n * sizeof(keto_tuple), hipMemcpyDeviceToDevice));
        buf = std::move(nb);
        reindex();
    }
    // every stored row entered afresh (a grown store, or tombstones past the load bound)
    void reindex() {
        const uint64_t slots = std::min<uint64_t>(0xFFFFFFFFull, cap() + cap() / 2 + 64);
        if (ix_slots != slots) {
            ix = build::DevBuf();
            ix = build::DevBuf(8 * slots);
            ix_slots = slots;
        }
        KETO_HIP(hipMemset(ix.p, 0xFF, 8 * slots));
        if (n) hipLaunchKernelGGL(k_ix_insert, grid_for(n), dim3(BLK), 0, 0, rows(), 0, n, index());
        KETO_HIP(hipGetLastError());
        if (getenv("KETO_PATCH_VERBOSE"))
            fprintf(stderr, "[keto store] index: %llu rows, %llu slots (%llu entries and tombstones before)\n", (unsigned long long)n,
                    (unsigned long long)slots, (unsigned long long)ix_used);
        ix_used = n;
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
    st->reindex();
    KETO_HIP(hipDeviceSynchronize());
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
    // tombstones and the new rows' entries within 3/4 of the index, or every row entered afresh
    // (amortised: a transaction of k rows spends k of the quarter's headroom)
    if ((st.ix_dirty || st.ix_used + n_ins > st.ix_slots / 4 * 3) && st.cap() >= st.n + n_ins) st.reindex();
    st.ix_dirty = true;  // (until the transaction is applied)
    if (n_ins) {  // WriteRelationTuples: appended rows, fresh shard_ids from the caller, indexed
        st.reserve(st.n + n_ins);  // (a grown store is indexed afresh, these rows not yet)
        KETO_HIP(hipMemcpy(st.rows() + st.n, ins, n_ins * sizeof(keto_tuple), kind));
        hipLaunchKernelGGL(k_ix_insert, grid_for(n_ins), dim3(BLK), 0, 0, st.rows(), n_before, n_ins, st.index());
        KETO_HIP(hipGetLastError());
        st.ix_used += n_ins;
    }
    // (the appended rows count only once the deletes below went through: st.n stays n_before
    // until the end.  A throw part-way leaves the index ahead of st.n: ix_dirty, and the next
    // transaction re-indexes first)
    const uint64_t n_all = n_before + n_ins;
    uint64_t n_after = n_all;
    if (n_del && n_all) {  // DeleteRelationTuples over everything, the new rows included
        build::DevBuf d(n_del * sizeof(keto_tuple)), cnt(8);
        KETO_HIP(hipMemcpy(d.p, del, n_del * sizeof(keto_tuple), kind));
        KETO_HIP(hipMemset(cnt.p, 0, 8));
        // (a delete key matches any number of rows: the dead list is sized by a first count)
        uint64_t cap_dead = std::max<uint64_t>(1024, 4 * n_del);
        unsigned long long n_dead = 0;
        build::DevBuf dead(4 * cap_dead);
        for (;;) {
            hipLaunchKernelGGL(k_ix_delete, grid_for(n_del), dim3(BLK), 0, 0, st.rows(), static_cast<const keto_tuple *>(d.p), n_del,
                               st.index(), dead.u32(), cap_dead, static_cast<unsigned long long *>(cnt.p));
            KETO_HIP(hipGetLastError());
            KETO_HIP(hipMemcpy(&n_dead, cnt.p, 8, hipMemcpyDeviceToHost));
            if (n_dead <= cap_dead) break;
            // more rows than the list held: the tombstoned ones are gone from the index already,
            // so the whole index is rebuilt from the rows and the deletes run again into a list
            // of the right size
            {  // (index every row, the appended ones included; st.n back to n_before on a throw too)
                struct Restore {
                    uint64_t &n, v;
                    ~Restore() { n = v; }
                } restore{st.n, n_before};
                st.n = n_all;
                st.reindex();
            }
            cap_dead = n_dead;
            dead = build::DevBuf(4 * cap_dead);
            KETO_HIP(hipMemset(cnt.p, 0, 8));
        }
        if (n_dead) {
            std::vector<uint32_t> dl(n_dead);
            KETO_HIP(hipMemcpy(dl.data(), dead.p, 4 * n_dead, hipMemcpyDeviceToHost));
            std::sort(dl.begin(), dl.end());
            const uint64_t keep = n_all - n_dead;
            // holes: dead positions below keep; movers: live positions at or above it (as many)
            std::vector<uint2> moves;
            size_t h = 0, dk = (size_t)(std::lower_bound(dl.begin(), dl.end(), (uint32_t)keep) - dl.begin());
            for (uint64_t p = keep; p < n_all; p++) {
                if (dk < dl.size() && dl[dk] == p) {
                    dk++;
                    continue;
                }
                moves.push_back(make_uint2((uint32_t)p, dl[h++]));
            }
            if (h != (size_t)(std::lower_bound(dl.begin(), dl.end(), (uint32_t)keep) - dl.begin()))
                throw Error(KETO_E_DEVICE, "compaction lists disagree");
            if (!moves.empty()) {
                build::DevBuf dm(sizeof(uint2) * moves.size());
                KETO_HIP(hipMemcpy(dm.p, moves.data(), sizeof(uint2) * moves.size(), hipMemcpyHostToDevice));
                hipLaunchKernelGGL(k_ix_move, grid_for(moves.size()), dim3(BLK), 0, 0, st.rows(), static_cast<const uint2 *>(dm.p),
                                   (uint64_t)moves.size(), st.index());
                KETO_HIP(hipGetLastError());
            }
            n_after = keep;
        }
    }
    KETO_HIP(hipDeviceSynchronize());
    // applied: the new content, its version and its log entry together
    st.n = n_after;
    st.ix_dirty = false;
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
