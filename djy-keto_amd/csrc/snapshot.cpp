// Snapshot builder: relation tuples + namespace AST -> device-resident CSR snapshot.
//
// Replaces the storage read path of the reference (internal/persistence/sql):
//   * set rows  = TraverseSubjectSetExpansion / GetRelationTuples restricted to
//                 subject sets, ORDER BY shard_id (traverser.go:68-92, relationtuples.go:216)
//   * all rows  = GetRelationTuples for Expand (expand/engine.go:84-95)
//   * rev rows  = ExistsRelationTuples / the EXISTS "found" lookahead / the OR
//                 computed-userset IN probe (relationtuples.go:249-261,
//                 traverser.go:73-80, 146-154): subject -> sorted nodes holding it
// and compiles the namespace AST (internal/namespace/ast) into a flat op table.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <numeric>
#include <thread>
#include <unordered_map>

#include "engine.hpp"
#include "json.hpp"

namespace keto {

namespace {

template <class T>
void parallel_sort(std::vector<T> &v) {
    const size_t n = v.size();
    unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1u << 20) || hw == 1) {
        std::sort(v.begin(), v.end());
        return;
    }
    size_t parts = 1;
    while (parts * 2 <= hw) parts *= 2;
    std::vector<size_t> bounds(parts + 1);
    for (size_t i = 0; i <= parts; i++) bounds[i] = n * i / parts;
    std::vector<std::thread> th;
    for (size_t i = 0; i < parts; i++)
        th.emplace_back([&, i] { std::sort(v.begin() + bounds[i], v.begin() + bounds[i + 1]); });
    for (auto &t : th) t.join();
    for (size_t w = 1; w < parts; w *= 2) {
        std::vector<std::thread> mt;
        for (size_t i = 0; i + w < parts; i += 2 * w) {
            size_t a = bounds[i], m = bounds[i + w], b = bounds[std::min(parts, i + 2 * w)];
            mt.emplace_back([&v, a, m, b] { std::inplace_merge(v.begin() + a, v.begin() + m, v.begin() + b); });
        }
        for (auto &t : mt) t.join();
    }
}

uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

struct Decl {
    uint32_t rel;
    uint32_t op;
    bool has_ss;
};

struct Compiler {
    Snapshot &s;
    std::unordered_map<std::string, uint32_t> rel_ids;

    uint32_t rel_id(const std::string &name) {
        auto it = rel_ids.find(name);
        if (it != rel_ids.end()) return it->second;
        uint32_t id = (uint32_t)s.rel_names.size();
        s.rel_names.push_back(name);
        rel_ids.emplace(name, id);
        return id;
    }

    static const std::string &str_field(const json::Value &v, const char *k) {
        const json::Value *f = v.get(k);
        if (!f || f->kind != json::Value::String)
            throw Error(KETO_E_INVALID, std::string("namespace JSON: expected string field '") + k + "'");
        return f->str;
    }

    // flattened ast.Child (ast_definitions.go:82-109)
    uint32_t compile(const json::Value &v) {
        if (v.kind != json::Value::Object) throw Error(KETO_E_INVALID, "namespace JSON: rewrite child must be an object");
        Op op{};
        if (v.has("operator") || v.has("children")) {
            uint32_t kind = OPK_OR;  // ast.OperatorOr is the zero value
            if (const json::Value *o = v.get("operator")) {
                if (o->kind == json::Value::String) kind = o->str == "or" ? OPK_OR : (o->str == "and" ? OPK_AND : OPK_BAD);
                else if (o->kind == json::Value::Number) kind = o->num == 0 ? OPK_OR : (o->num == 1 ? OPK_AND : OPK_BAD);
                else kind = OPK_BAD;
            }
            std::vector<uint32_t> kids;
            bool has_css = false;
            if (const json::Value *c = v.get("children")) {
                if (c->kind == json::Value::Array)
                    for (auto &ch : c->arr) {
                        uint32_t k = compile(ch);
                        kids.push_back(k);
                        if ((s.ops[k].type_kind & 0xFF) == OP_CSS) has_css = true;
                    }
            }
            op.type_kind = OP_REWRITE | (kind << 8) | (uint32_t(has_css) << 16);
            op.child_begin = (uint32_t)s.op_children.size();
            op.child_count = (uint32_t)kids.size();
            s.op_children.insert(s.op_children.end(), kids.begin(), kids.end());
        } else if (const json::Value *inv = v.get("inverted")) {
            uint32_t k = compile(*inv);
            op.type_kind = OP_INVERT;
            op.child_begin = (uint32_t)s.op_children.size();
            op.child_count = 1;
            s.op_children.push_back(k);
        } else if (v.has("computed_subject_set_relation")) {
            op.type_kind = OP_TTU;
            op.rel_computed = rel_id(str_field(v, "relation")) | (rel_id(str_field(v, "computed_subject_set_relation")) << 16);
        } else if (v.has("relation")) {
            op.type_kind = OP_CSS;
            op.rel_computed = rel_id(str_field(v, "relation"));
        } else {
            throw Error(KETO_E_INVALID, "namespace JSON: unknown rewrite child");
        }
        if (s.ops.size() >= NO_OP) throw Error(KETO_E_LIMIT, "rewrite program exceeds 65535 ops");
        s.ops.push_back(op);
        return (uint32_t)s.ops.size() - 1;
    }
};

template <class T>
T *upload(Snapshot &s, const std::vector<T> &v, size_t min_elems = 1) {
    // padded to 16 bytes (+16) so 16-byte window loads past the end stay in bounds
    size_t bytes = (std::max(v.size(), min_elems) * sizeof(T) + 31) / 16 * 16;
    void *p = nullptr;
    KETO_HIP(hipMalloc(&p, bytes));
    s.allocs.push_back(p);
    KETO_HIP(hipMemset(p, 0, bytes));
    if (!v.empty()) KETO_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    s.info.device_bytes += bytes;
    return static_cast<T *>(p);
}

template <class T>
uint32_t bytes16(const std::vector<T> &v) {
    return (uint32_t)((v.size() * sizeof(T) + 15) / 16 * 16);
}

}  // namespace

Snapshot::~Snapshot() {
    for (void *p : allocs) (void)hipFree(p);
}

uint32_t Snapshot::ns_of(uint32_t node) const {
    // last ns with node_base <= node (empty namespaces share bases; take the last)
    uint32_t lo = 0, hi = n_ns;
    while (lo + 1 < hi) {
        uint32_t m = (lo + hi) / 2;
        if (ns[m].node_base <= node) lo = m;
        else hi = m;
    }
    while (lo + 1 < n_ns && ns[lo + 1].node_base <= node) lo++;
    return lo;
}

Snapshot *build_snapshot(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n) {
    auto t0 = std::chrono::steady_clock::now();
    if (!cfg) throw Error(KETO_E_INVALID, "null config");
    if (n && !tuples) throw Error(KETO_E_INVALID, "null tuples");
    if (cfg->n_namespaces == 0 || cfg->n_namespaces > 0x7FFF)
        throw Error(KETO_E_LIMIT, "n_namespaces must be in [1, 32767]");
    if (cfg->n_uuids >= 0x80000000u) throw Error(KETO_E_LIMIT, "n_uuids must be < 2^31");
    KETO_HIP(hipSetDevice(cfg->device));

    auto S = std::make_unique<Snapshot>();
    Snapshot &s = *S;
    s.device = cfg->device;
    s.n_ns = cfg->n_namespaces;
    s.n_uuids = cfg->n_uuids;
    s.strict = cfg->strict_mode != 0;
    s.n_rel_caller = cfg->n_relations;
    Compiler C{s, {}};
    for (uint32_t i = 0; i < s.n_ns; i++) s.ns_names.emplace_back(cfg->namespace_names && cfg->namespace_names[i] ? cfg->namespace_names[i] : "");
    for (uint32_t i = 0; i < cfg->n_relations; i++) {
        std::string nm = cfg->relation_names && cfg->relation_names[i] ? cfg->relation_names[i] : "";
        s.rel_names.push_back(nm);
        C.rel_ids.emplace(nm, i);  // first id wins for duplicate names
    }
    std::unordered_map<std::string, uint32_t> ns_ids;
    for (uint32_t i = 0; i < s.n_ns; i++) ns_ids.emplace(s.ns_names[i], i);

    // ---- namespace AST ------------------------------------------------------
    std::vector<uint8_t> configured(s.n_ns, 0);
    std::vector<std::vector<Decl>> decls(s.n_ns);
    if (cfg->namespaces_json && cfg->namespaces_json[0]) {
        json::Value root;
        try {
            root = json::parse(cfg->namespaces_json);
        } catch (const std::exception &e) {
            throw Error(KETO_E_INVALID, e.what());
        }
        if (root.kind != json::Value::Object) throw Error(KETO_E_INVALID, "namespace JSON must be an object {ns: [relations]}");
        for (auto &kv : root.obj) {
            auto it = ns_ids.find(kv.first);
            if (kv.second.kind != json::Value::Array && kv.second.kind != json::Value::Null)
                throw Error(KETO_E_INVALID, "namespace JSON: relations of '" + kv.first + "' must be a list");
            std::vector<Decl> ds;
            for (auto &r : kv.second.arr) {
                Decl d{C.rel_id(Compiler::str_field(r, "name")), NO_OP, false};
                if (const json::Value *ty = r.get("types"))
                    for (auto &t : ty->arr)
                        if (const json::Value *tr = t.get("relation"))
                            if (tr->kind == json::Value::String && !tr->str.empty()) d.has_ss = true;  // engine.go:251-258
                if (const json::Value *rw = r.get("rewrite"))
                    if (rw->kind != json::Value::Null) d.op = C.compile(*rw);
                ds.push_back(d);
            }
            if (it == ns_ids.end()) continue;  // never referenced by a tuple or query id
            configured[it->second] = 1;
            decls[it->second] = std::move(ds);
        }
    }
    s.n_rel = (uint32_t)s.rel_names.size();
    if (s.n_rel >= 0xFFFF) throw Error(KETO_E_LIMIT, "more than 65534 relation names");
    int64_t empty_rel = -1;
    {
        auto it = C.rel_ids.find("");
        if (it != C.rel_ids.end()) empty_rel = it->second;
    }

    // ---- validate tuples, collect (ns, rel) pairs ------------------------------
    const size_t NR = (size_t)s.n_ns * s.n_rel;
    if (NR > (1ull << 28)) throw Error(KETO_E_LIMIT, "n_namespaces * n_relations too large");
    std::vector<uint8_t> used(NR, 0);
    for (uint64_t i = 0; i < n; i++) {
        const keto_tuple &t = tuples[i];
        if (t.ns >= s.n_ns || t.rel >= s.n_rel_caller || t.obj >= s.n_uuids || t.s_obj >= s.n_uuids || t.subj_kind > 1 ||
            (t.subj_kind == 1 && (t.s_ns >= s.n_ns || t.s_rel >= s.n_rel_caller)))
            throw Error(KETO_E_INVALID, "tuple " + std::to_string(i) + " has an out-of-range id");
        used[(size_t)t.ns * s.n_rel + t.rel] = 1;
        if (t.subj_kind == 1) used[(size_t)t.s_ns * s.n_rel + t.s_rel] = 1;
    }

    // ---- relation slots + status (namespace.ASTRelationFor, definitions.go:37-62) -------
    s.nsrel.assign(NR, 0);
    s.ns.resize(s.n_ns + 1);
    std::vector<uint32_t> slot_of(NR, NO_SLOT);
    uint32_t total_slots = 0;
    for (uint32_t ns = 0; ns < s.n_ns; ns++) {
        std::vector<uint32_t> rels;
        std::vector<uint8_t> has(s.n_rel, 0);
        for (auto &d : decls[ns])
            if (!has[d.rel]) {
                has[d.rel] = 1;
                rels.push_back(d.rel);
            }
        for (uint32_t r = 0; r < s.n_rel; r++)
            if (used[(size_t)ns * s.n_rel + r] && !has[r]) {
                has[r] = 1;
                rels.push_back(r);
            }
        if (rels.size() >= NO_SLOT) throw Error(KETO_E_LIMIT, "namespace with more than 65534 relations");
        s.ns[ns].slot_base = total_slots;
        s.ns[ns].n_slots = (uint32_t)rels.size();
        for (uint32_t k = 0; k < rels.size(); k++) slot_of[(size_t)ns * s.n_rel + rels[k]] = k;
        for (uint32_t r : rels) s.slot_rel.push_back(r);
        total_slots += (uint32_t)rels.size();
        for (uint32_t r = 0; r < s.n_rel; r++) {
            uint32_t status;
            const Decl *decl = nullptr;
            if ((int64_t)r == empty_rel || !configured[ns] || decls[ns].empty()) status = REL_NIL;
            else {
                for (auto &d : decls[ns])
                    if (d.rel == r) {
                        decl = &d;
                        break;
                    }
                status = decl ? REL_DECLARED : REL_ERROR;
            }
            s.nsrel[(size_t)ns * s.n_rel + r] = slot_of[(size_t)ns * s.n_rel + r] | (status << 16);
        }
    }
    s.relinfo.resize(total_slots);
    for (uint32_t ns = 0; ns < s.n_ns; ns++)
        for (uint32_t k = 0; k < s.ns[ns].n_slots; k++) {
            uint32_t r = s.slot_rel[s.ns[ns].slot_base + k];
            uint32_t status = nr_status(s.nsrel[(size_t)ns * s.n_rel + r]);
            const Decl *decl = nullptr;
            if (status == REL_DECLARED)
                for (auto &d : decls[ns])
                    if (d.rel == r) {
                        decl = &d;
                        break;
                    }
            bool rw = decl && decl->op != NO_OP;
            bool ss = !s.strict || !decl || decl->has_ss;  // engine.go:235
            s.relinfo[s.ns[ns].slot_base + k] = make_ri(rw ? decl->op : NO_OP, rw, ss, status, false);
        }

    // ---- entities: (ns, obj) of tuple objects and subject-set objects -----------------
    std::vector<uint64_t> ek;
    ek.reserve(n + n / 2);
    for (uint64_t i = 0; i < n; i++) {
        ek.push_back(((uint64_t)tuples[i].ns << 32) | tuples[i].obj);
        if (tuples[i].subj_kind == 1) ek.push_back(((uint64_t)tuples[i].s_ns << 32) | tuples[i].s_obj);
    }
    parallel_sort(ek);
    ek.erase(std::unique(ek.begin(), ek.end()), ek.end());
    std::vector<uint32_t> n_real(s.n_ns, 0);
    for (uint64_t k : ek) n_real[k >> 32]++;
    uint64_t ent_total = 0, node_total = 0;
    for (uint32_t ns = 0; ns < s.n_ns; ns++) {
        s.ns[ns].ent_base = (uint32_t)ent_total;
        s.ns[ns].node_base = (uint32_t)node_total;
        uint64_t ne = (uint64_t)n_real[ns] + 1;  // + phantom
        ent_total += ne;
        node_total += ne * s.ns[ns].n_slots;
        if (node_total >= VIRT_BIT || ent_total >= VIRT_BIT) throw Error(KETO_E_LIMIT, "node space exceeds 2^31");
    }
    s.ns[s.n_ns] = NsDev{(uint32_t)ent_total, (uint32_t)node_total, 0, total_slots};
    const uint32_t N = (uint32_t)node_total;
    if ((uint64_t)s.n_uuids + N + 1 >= (1ull << 32)) throw Error(KETO_E_LIMIT, "n_uuids + nodes exceeds 2^32");
    s.ent_obj.assign(ent_total, NONE32);
    // entity hash: ((ns<<32)|obj)+1 -> entity
    uint64_t cap = 16;
    while (cap < 2 * ek.size() + 2) cap <<= 1;
    std::vector<unsigned long long> ent_keys(cap, 0);
    std::vector<uint32_t> ent_vals(cap, 0);  // host lookup copies; device gets 16-byte slots
    {
        std::vector<uint32_t> fill(s.n_ns, 0);
        for (uint64_t k : ek) {
            uint32_t ns = (uint32_t)(k >> 32);
            uint32_t e = s.ns[ns].ent_base + fill[ns]++;
            s.ent_obj[e] = (uint32_t)k;
            uint64_t h = mix64(k + 1) & (cap - 1);
            while (ent_keys[h]) h = (h + 1) & (cap - 1);
            ent_keys[h] = k + 1;
            ent_vals[h] = e;
        }
    }
    auto ent_lookup = [&](uint32_t ns, uint32_t obj) -> uint32_t {
        uint64_t key = (((uint64_t)ns << 32) | obj) + 1;
        uint64_t h = mix64(key) & (cap - 1);
        while (ent_keys[h]) {
            if (ent_keys[h] == key) return ent_vals[h];
            h = (h + 1) & (cap - 1);
        }
        return NONE32;
    };
    auto node_of = [&](uint32_t ns, uint32_t e, uint32_t rel) -> uint32_t {
        uint32_t slot = slot_of[(size_t)ns * s.n_rel + rel];
        return s.ns[ns].node_base + (e - s.ns[ns].ent_base) * s.ns[ns].n_slots + slot;
    };

    // ---- shard order rank (ORDER BY shard_id, UUID bytes big-endian) --------------------
    std::vector<uint32_t> src(n), dst(n), rank(n);
    {
        struct SK {
            uint64_t hi, lo;
            uint32_t idx;
            bool operator<(const SK &o) const { return hi != o.hi ? hi < o.hi : (lo != o.lo ? lo < o.lo : idx < o.idx); }
        };
        std::vector<SK> sk(n);
        for (uint64_t i = 0; i < n; i++) {
            uint64_t hi = 0, lo = 0;
            for (int b = 0; b < 8; b++) hi = (hi << 8) | tuples[i].shard_id[b];
            for (int b = 8; b < 16; b++) lo = (lo << 8) | tuples[i].shard_id[b];
            sk[i] = SK{hi, lo, (uint32_t)i};
        }
        parallel_sort(sk);
        for (uint64_t r = 0; r < n; r++) rank[sk[r].idx] = (uint32_t)r;
    }
    for (uint64_t i = 0; i < n; i++) {
        const keto_tuple &t = tuples[i];
        src[i] = node_of(t.ns, ent_lookup(t.ns, t.obj), t.rel);
        dst[i] = t.subj_kind == 1 ? node_of(t.s_ns, ent_lookup(t.s_ns, t.s_obj), t.s_rel) : t.s_obj;
    }

    // ---- rows: (node, shard rank) sorted ----------------------------------------------
    std::vector<uint32_t> by_rank(n);
    for (uint64_t i = 0; i < n; i++) by_rank[rank[i]] = (uint32_t)i;
    std::vector<uint32_t> set_off(N + 1, 0), all_off(N + 1, 0), set_dst, all_subj;
    {
        std::vector<uint64_t> keys;
        keys.reserve(n);
        for (uint64_t i = 0; i < n; i++) keys.push_back(((uint64_t)src[i] << 32) | rank[i]);
        parallel_sort(keys);
        all_subj.resize(n);
        uint64_t n_set = 0;
        for (uint64_t i = 0; i < n; i++) n_set += tuples[i].subj_kind == 1;
        set_dst.resize(n_set);
        uint64_t si = 0;
        for (uint64_t i = 0; i < n; i++) {
            uint32_t node = (uint32_t)(keys[i] >> 32);
            uint32_t ti = by_rank[(uint32_t)keys[i]];
            all_off[node + 1]++;
            bool is_set = tuples[ti].subj_kind == 1;
            all_subj[i] = is_set ? (SKEY_SET | dst[ti]) : dst[ti];
            if (is_set) {
                set_off[node + 1]++;
                set_dst[si++] = dst[ti];
            }
        }
        for (uint32_t v = 0; v < N; v++) {
            all_off[v + 1] += all_off[v];
            set_off[v + 1] += set_off[v];
        }
        if (n >= (1ull << 32)) throw Error(KETO_E_LIMIT, "more than 2^32 tuples");
    }

    // ---- reverse membership rows: subject -> sorted nodes ---------------------------------
    const uint64_t n_subj_idx = (uint64_t)s.n_uuids + N;
    std::vector<uint32_t> rev_off(n_subj_idx + 1, 0), rev_nodes;
    {
        std::vector<uint64_t> keys(n);
        for (uint64_t i = 0; i < n; i++) {
            uint64_t idx = tuples[i].subj_kind == 1 ? (uint64_t)s.n_uuids + dst[i] : dst[i];
            keys[i] = (idx << 32) | src[i];
        }
        parallel_sort(keys);
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        rev_nodes.resize(keys.size());
        for (size_t i = 0; i < keys.size(); i++) {
            rev_off[(keys[i] >> 32) + 1]++;
            rev_nodes[i] = (uint32_t)keys[i];
        }
        for (uint64_t v = 0; v < n_subj_idx; v++) rev_off[v + 1] += rev_off[v];
    }

    // ---- visited keys: UUIDv5(obj, ns+"-"+rel) (relationtuple/definitions.go:114-116) -------
    std::vector<uint32_t> vkey;
    {
        std::unordered_map<std::string, std::vector<uint32_t>> cls;  // class string -> global slots
        for (uint32_t ns = 0; ns < s.n_ns; ns++)
            for (uint32_t k = 0; k < s.ns[ns].n_slots; k++)
                cls[s.ns_names[ns] + "-" + s.rel_names[s.slot_rel[s.ns[ns].slot_base + k]]].push_back(s.ns[ns].slot_base + k);
        bool any_shared = false;
        for (auto &kv : cls)
            if (kv.second.size() > 1) any_shared = true;
        if (any_shared) {
            vkey.resize(N);
            std::iota(vkey.begin(), vkey.end(), 0u);
            std::vector<uint32_t> slot_ns(total_slots);
            for (uint32_t ns = 0; ns < s.n_ns; ns++)
                for (uint32_t k = 0; k < s.ns[ns].n_slots; k++) slot_ns[s.ns[ns].slot_base + k] = ns;
            for (auto &kv : cls) {
                if (kv.second.size() < 2) continue;
                std::unordered_map<uint32_t, uint32_t> rep;  // obj -> min node
                std::vector<uint32_t> members;
                for (uint32_t gs : kv.second) {
                    uint32_t ns = slot_ns[gs], k = gs - s.ns[ns].slot_base;
                    s.relinfo[gs] |= 1u << 20;
                    uint32_t real = n_real[ns];
                    for (uint32_t j = 0; j < real; j++) {
                        uint32_t e = s.ns[ns].ent_base + j;
                        uint32_t node = s.ns[ns].node_base + j * s.ns[ns].n_slots + k;
                        auto it = rep.find(s.ent_obj[e]);
                        if (it == rep.end()) rep.emplace(s.ent_obj[e], node);
                        else it->second = std::min(it->second, node);
                        members.push_back(node);
                    }
                }
                for (uint32_t node : members) {
                    uint32_t ns = s.ns_of(node);
                    uint32_t e = s.ns[ns].ent_base + (node - s.ns[ns].node_base) / s.ns[ns].n_slots;
                    vkey[node] = rep[s.ent_obj[e]];
                }
            }
            for (auto &d : set_dst)
                if (vkey[d] != d) d |= EDGE_ALIAS;
        }
    }

    // ---- upload ------------------------------------------------------------------------
    DevSnapshot &D = s.dev;
    {
        std::vector<uint32_t> set_row(2 * (size_t)N);
        for (uint32_t v = 0; v < N; v++) {
            set_row[2 * v] = set_off[v];
            set_row[2 * v + 1] = set_off[v + 1];
        }
        D.set_row = upload(s, set_row);
        // capped count of expansion paths below each node (relaxed to a fixed point over
        // WEIGHT_ROUNDS rounds): a cost estimate that orders each batch longest-first
        std::vector<uint32_t> wgt(N, 1), nxt(N);
        for (int round = 0; round < WEIGHT_ROUNDS; round++) {
            for (uint32_t v = 0; v < N; v++) {
                uint64_t acc = 1;
                for (uint32_t i = set_off[v]; i < set_off[v + 1] && acc < WEIGHT_CAP; i++) acc += wgt[set_dst[i] & ~EDGE_ALIAS];
                nxt[v] = (uint32_t)std::min<uint64_t>(acc, WEIGHT_CAP);
            }
            wgt.swap(nxt);
        }
        D.weight = upload(s, wgt);
    }
    D.set_dst = upload(s, set_dst);
    D.vkey = vkey.empty() ? nullptr : upload(s, vkey);
    D.all_off = upload(s, all_off);
    D.all_subj = upload(s, all_subj);
    D.rev_off = upload(s, rev_off);
    D.rev_nodes = upload(s, rev_nodes);
    D.ns = upload(s, s.ns);
    D.relinfo = upload(s, s.relinfo);
    D.nsrel = upload(s, s.nsrel);
    D.ops = upload(s, s.ops);
    D.op_children = upload(s, s.op_children);
    D.tab_bytes[0] = bytes16(s.ns);
    D.tab_bytes[1] = bytes16(s.relinfo);
    D.tab_bytes[2] = bytes16(s.nsrel);
    D.tab_bytes[3] = bytes16(s.ops);
    D.tab_bytes[4] = bytes16(s.op_children);
    D.lds_bytes = 0;
    for (uint32_t b : D.tab_bytes) D.lds_bytes += b;
    {
        std::vector<uint32_t> et(4 * cap, 0);
        for (uint64_t i = 0; i < cap; i++) {
            et[4 * i + 0] = (uint32_t)ent_keys[i];
            et[4 * i + 1] = (uint32_t)(ent_keys[i] >> 32);
            et[4 * i + 2] = ent_vals[i];
        }
        D.ent_table = reinterpret_cast<const uint4 *>(upload(s, et));
        D.ent_mask = (uint32_t)(cap - 1);
    }
    // membership probe hash for subjects whose reverse row exceeds PROBE_K
    {
        uint64_t heavy = 0;
        for (uint64_t v = 0; v < n_subj_idx; v++)
            if (rev_off[v + 1] - rev_off[v] > PROBE_K) heavy += rev_off[v + 1] - rev_off[v];
        uint64_t buckets = 1;
        while (buckets * 2 < heavy * 2 + 2) buckets <<= 1;  // load factor <= 1/2
        std::vector<uint64_t> pt(2 * buckets, 0);
        for (uint64_t v = 0; v < n_subj_idx; v++) {
            if (rev_off[v + 1] - rev_off[v] <= PROBE_K) continue;
            for (uint32_t i = rev_off[v]; i < rev_off[v + 1]; i++) {
                uint64_t key = ((v << 32) | rev_nodes[i]) + 1;
                uint64_t b = mix64(key) & (buckets - 1);
                while (true) {
                    if (!pt[2 * b]) {
                        pt[2 * b] = key;
                        break;
                    }
                    if (!pt[2 * b + 1]) {
                        pt[2 * b + 1] = key;
                        break;
                    }
                    b = (b + 1) & (buckets - 1);
                }
            }
        }
        D.probe = reinterpret_cast<const uint4 *>(upload(s, pt));
        D.probe_mask = (uint32_t)(buckets - 1);
        D.probe_k = PROBE_K;
    }
    D.n_ns = s.n_ns;
    D.n_rel = s.n_rel;
    D.n_nodes = N;
    D.n_uuids = s.n_uuids;
    D.strict = s.strict;

    s.info.n_tuples = n;
    s.info.n_nodes = N;
    s.info.n_entities = ent_total;
    s.info.n_set_edges = set_dst.size();
    s.info.n_rev_entries = rev_nodes.size();
    s.info.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return S.release();
}

}  // namespace keto
