// Expand trees -> API form: the host-side batched pass the shim
// runs after keto_expand_batch.
//
//   Mapper.ToTree        internal/relationtuple/uuid_mapping.go:347-399
//     ids -> strings: namespace name, UUID -> string (MapUUIDsToStrings), relation as stored.
//     Each node's tuple carries only its subject (namespace/object/relation stay "").
//   encoding/json of ketoapi.Tree[*RelationTuple]   ketoapi/public_api_definitions.go:217-229
//     {"type", "children" (omitempty), "tuple"}; RelationTuple {"namespace", "object",
//     "relation", "subject_id" | "subject_set"} (:35-62).  json.Marshal's default string
//     escaping (HTML-safe <, >, & ; U+2028/9; invalid UTF-8 -> U+FFFD; go.mod pins go 1.21,
//     so control characters other than \n \r \t are \u00XX).
//   Tree.ToProto          ketoapi/enc_proto.go:119-133
//     SubjectTree {node_type = 1, subject = 2 (deprecated copy of tuple.subject),
//     children = 3, tuple = 4}; wire order by field number, proto3 default values omitted,
//     the Subject oneof always present (expand_service.proto:64-92,
//     relation_tuples.proto:13-74).
#include <cstring>
#include <string>
#include <vector>

#include "engine.hpp"

namespace keto {
namespace {

constexpr uint32_t T_UNION = 1, T_EXCLUSION = 2, T_INTERSECTION = 3, T_LEAF = 4;

const char *type_name(uint32_t t) {
    switch (t) {
        case T_UNION: return "union";
        case T_EXCLUSION: return "exclusion";
        case T_INTERSECTION: return "intersection";
        case T_LEAF: return "leaf";
        default: return "unspecified";
    }
}

struct Names {
    const keto_name_tables *t;
    const char *ns(uint32_t i) const {
        if (i >= t->n_namespaces) throw Error(KETO_E_INVALID, "tree names an unknown namespace id");
        return t->namespace_names[i];
    }
    const char *rel(uint32_t i) const {
        if (i >= t->n_relations) throw Error(KETO_E_INVALID, "tree names an unknown relation id");
        return t->relation_names[i];
    }
    const char *uuid(uint32_t i) const {
        if (i >= t->n_uuids) throw Error(KETO_E_INVALID, "tree names an unknown object id");
        return t->uuid_strings[i];
    }
};

// ---- JSON ------------------------------------------------------------------------------

void json_str(std::string &o, const char *s) {
    static const char *hex = "0123456789abcdef";
    o += '"';
    const auto *p = reinterpret_cast<const unsigned char *>(s);
    while (*p) {
        const unsigned char c = *p;
        if (c < 0x80) {
            if (c == '"' || c == '\\') {
                o += '\\';
                o += (char)c;
            } else if (c == '\n') {
                o += "\\n";
            } else if (c == '\r') {
                o += "\\r";
            } else if (c == '\t') {
                o += "\\t";
            } else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                o += "\\u00";
                o += hex[c >> 4];
                o += hex[c & 15];
            } else {
                o += (char)c;
            }
            p++;
            continue;
        }
        // one UTF-8 sequence, validated as Go's utf8.DecodeRuneInString does
        int len = 0;
        uint32_t cp = 0;
        if (c >= 0xC2 && c <= 0xDF) len = 2, cp = c & 0x1F;
        else if (c >= 0xE0 && c <= 0xEF) len = 3, cp = c & 0x0F;
        else if (c >= 0xF0 && c <= 0xF4) len = 4, cp = c & 0x07;
        bool ok = len > 0;
        for (int k = 1; ok && k < len; k++) {
            if ((p[k] & 0xC0) != 0x80) ok = false;
            else cp = (cp << 6) | (p[k] & 0x3F);
        }
        if (ok && ((len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF))))
            ok = false;
        if (!ok) {
            o += "\\ufffd";
            p++;
            continue;
        }
        if (cp == 0x2028 || cp == 0x2029) {
            o += cp == 0x2028 ? "\\u2028" : "\\u2029";
        } else {
            o.append(reinterpret_cast<const char *>(p), len);
        }
        p += len;
    }
    o += '"';
}

// subtree sizes (in nodes) of a pre-order tree, checked for consistency
std::vector<uint64_t> subtree_counts(const keto_tree_node *n, uint64_t m) {
    std::vector<uint64_t> cnt(m, 0);
    for (uint64_t i = m; i-- > 0;) {
        uint64_t c = 1, j = i + 1;
        for (uint32_t k = 0; k < n[i].n_children; k++) {
            if (j >= m) throw Error(KETO_E_INVALID, "malformed pre-order tree");
            c += cnt[j];
            j += cnt[j];
        }
        cnt[i] = c;
    }
    if (m && cnt[0] != m) throw Error(KETO_E_INVALID, "malformed pre-order tree");
    return cnt;
}

void json_node(std::string &o, const keto_tree_node *n, uint64_t i, const std::vector<uint64_t> &cnt,
               const Names &nm) {
    o += "{\"type\":";
    json_str(o, type_name(n[i].type));
    if (n[i].n_children) {
        o += ",\"children\":[";
        uint64_t j = i + 1;
        for (uint32_t k = 0; k < n[i].n_children; k++) {
            if (k) o += ',';
            json_node(o, n, j, cnt, nm);
            j += cnt[j];
        }
        o += ']';
    }
    o += ",\"tuple\":{\"namespace\":\"\",\"object\":\"\",\"relation\":\"\",";
    if (n[i].subj_kind == 1) {
        o += "\"subject_set\":{\"namespace\":";
        json_str(o, nm.ns(n[i].s_ns));
        o += ",\"object\":";
        json_str(o, nm.uuid(n[i].s_obj));
        o += ",\"relation\":";
        json_str(o, nm.rel(n[i].s_rel));
        o += '}';
    } else {
        o += "\"subject_id\":";
        json_str(o, nm.uuid(n[i].s_obj));
    }
    o += "}}";
}

// ---- protobuf wire format ---------------------------------------------------------------

uint64_t varint_len(uint64_t v) {
    uint64_t l = 1;
    while (v >= 0x80) v >>= 7, l++;
    return l;
}
void put_varint(std::string &o, uint64_t v) {
    while (v >= 0x80) {
        o += (char)(uint8_t)(v | 0x80);
        v >>= 7;
    }
    o += (char)(uint8_t)v;
}
// length-delimited field: tag, length, payload
uint64_t ld_len(uint64_t payload) { return 1 + varint_len(payload) + payload; }
void put_ld(std::string &o, uint32_t field, const char *s, uint64_t len) {
    put_varint(o, (uint64_t)field << 3 | 2);
    put_varint(o, len);
    o.append(s, len);
}
void put_str_nonempty(std::string &o, uint32_t field, const char *s) {  // proto3: "" omitted
    const uint64_t l = std::strlen(s);
    if (l) put_ld(o, field, s, l);
}
uint64_t str_nonempty_len(const char *s) {
    const uint64_t l = std::strlen(s);
    return l ? ld_len(l) : 0;
}

// Subject {oneof ref: id = 1 | set = 2 (SubjectSet {namespace 1, object 2, relation 3})}
uint64_t subject_set_len(const keto_tree_node &x, const Names &nm) {
    return str_nonempty_len(nm.ns(x.s_ns)) + str_nonempty_len(nm.uuid(x.s_obj)) + str_nonempty_len(nm.rel(x.s_rel));
}
uint64_t subject_len(const keto_tree_node &x, const Names &nm) {
    if (x.subj_kind == 1) return ld_len(subject_set_len(x, nm));
    return ld_len(std::strlen(nm.uuid(x.s_obj)));  // a oneof member is present even if ""
}
void put_subject(std::string &o, const keto_tree_node &x, const Names &nm) {
    if (x.subj_kind == 1) {
        put_varint(o, 2u << 3 | 2);
        put_varint(o, subject_set_len(x, nm));
        put_str_nonempty(o, 1, nm.ns(x.s_ns));
        put_str_nonempty(o, 2, nm.uuid(x.s_obj));
        put_str_nonempty(o, 3, nm.rel(x.s_rel));
    } else {
        const char *id = nm.uuid(x.s_obj);
        put_ld(o, 1, id, std::strlen(id));
    }
}

// SubjectTree: node_type 1 (varint), subject 2, children 3 (repeated), tuple 4
//   (RelationTuple: namespace/object/relation "" -> omitted, subject = 4)
std::vector<uint64_t> proto_sizes(const keto_tree_node *n, uint64_t m, const std::vector<uint64_t> &cnt,
                                  const Names &nm) {
    std::vector<uint64_t> sz(m, 0);
    for (uint64_t i = m; i-- > 0;) {
        const uint64_t subj = subject_len(n[i], nm);
        uint64_t s = (n[i].type ? 1 + varint_len(n[i].type) : 0) + ld_len(subj) + ld_len(ld_len(subj));
        uint64_t j = i + 1;
        for (uint32_t k = 0; k < n[i].n_children; k++) {
            s += ld_len(sz[j]);
            j += cnt[j];
        }
        sz[i] = s;
    }
    return sz;
}

void proto_node(std::string &o, const keto_tree_node *n, uint64_t i, const std::vector<uint64_t> &cnt,
                const std::vector<uint64_t> &sz, const Names &nm) {
    if (n[i].type) {
        put_varint(o, 1u << 3 | 0);
        put_varint(o, n[i].type);
    }
    const uint64_t subj = subject_len(n[i], nm);
    put_varint(o, 2u << 3 | 2);  // deprecated SubjectTree.subject = tuple.subject
    put_varint(o, subj);
    put_subject(o, n[i], nm);
    uint64_t j = i + 1;
    for (uint32_t k = 0; k < n[i].n_children; k++) {
        put_varint(o, 3u << 3 | 2);
        put_varint(o, sz[j]);
        proto_node(o, n, j, cnt, sz, nm);
        j += cnt[j];
    }
    put_varint(o, 4u << 3 | 2);  // tuple {subject = 4}
    put_varint(o, ld_len(subj));
    put_varint(o, 4u << 3 | 2);
    put_varint(o, subj);
    put_subject(o, n[i], nm);
}

template <class F>
void format_batch(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees, char *out, uint64_t cap,
                  uint64_t *out_offsets, F one) {
    if (!offsets || !out_offsets || (n_trees && !nodes)) throw Error(KETO_E_INVALID, "null argument");
    uint64_t pos = 0;
    bool fits = true;
    std::string buf;
    for (uint64_t t = 0; t < n_trees; t++) {
        out_offsets[t] = pos;
        if (offsets[t + 1] < offsets[t]) throw Error(KETO_E_INVALID, "offsets must be non-decreasing");
        buf.clear();
        const uint64_t m = offsets[t + 1] - offsets[t];
        if (m) one(buf, nodes + offsets[t], m);  // an empty range is a nil tree: no bytes
        if (fits && pos + buf.size() <= cap && out) std::memcpy(out + pos, buf.data(), buf.size());
        else fits = false;
        pos += buf.size();
    }
    out_offsets[n_trees] = pos;
    if (!fits) throw Error(KETO_E_CAPACITY, "output buffer too small (out_offsets[n] = bytes required)");
}

}  // namespace

void trees_to_json(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                   const keto_name_tables *names, char *out, uint64_t cap, uint64_t *out_offsets) {
    if (!names) throw Error(KETO_E_INVALID, "null name tables");
    const Names nm{names};
    format_batch(nodes, offsets, n_trees, out, cap, out_offsets, [&](std::string &o, const keto_tree_node *n, uint64_t m) {
        const auto cnt = subtree_counts(n, m);
        json_node(o, n, 0, cnt, nm);
    });
}

void trees_to_proto(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                    const keto_name_tables *names, uint8_t *out, uint64_t cap, uint64_t *out_offsets) {
    if (!names) throw Error(KETO_E_INVALID, "null name tables");
    const Names nm{names};
    format_batch(nodes, offsets, n_trees, reinterpret_cast<char *>(out), cap, out_offsets,
                 [&](std::string &o, const keto_tree_node *n, uint64_t m) {
                     const auto cnt = subtree_counts(n, m);
                     const auto sz = proto_sizes(n, m, cnt, nm);
                     proto_node(o, n, 0, cnt, sz, nm);
                 });
}

}  // namespace keto
