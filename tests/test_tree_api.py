"""Expand trees -> API form (keto_trees_to_json / keto_trees_to_proto, csrc/treefmt.cpp):
host-only code, so it runs without a GPU.  The trees are built by the oracle; the oracle's
tree records have the same layout as keto_tree_node."""
import json
import os

import numpy as np
import pytest
from google.protobuf import descriptor_pb2, descriptor_pool, json_format, message_factory

import keto_mi355x as km
import refsem
from fixtures import GOLDEN, load, world_for
from keto_mi355x import api


def _beach():
    fx = load("docs_expand_beach")
    w, t, _ = world_for(fx)
    orc = refsem.Oracle(w, t)
    e = fx["expands"][0]
    ns, obj, rel = refsem.parse_subject_set(e["subject"])
    nodes, _ = orc.expand(1, w.uuids.ids[obj], w.ns_names.ids[ns], w.rel_names.ids[rel], e["depth"])
    names = api.NameTables(w.ns_names.names, w.rel_names.names, w.uuids.names)
    return w, nodes.view(km.TREE_DT), names


def _canon(tree):
    """order-insensitive form: children sorted by their canonical JSON"""
    t = dict(tree)
    if "children" in t:
        t["children"] = sorted((_canon(c) for c in t["children"]), key=lambda c: json.dumps(c, sort_keys=True))
    return t


def test_json_matches_docs_expected_output():
    _, nodes, names = _beach()
    out = api.trees_to_json(nodes, np.array([0, len(nodes)], np.uint64), names)
    with open(os.path.join(GOLDEN, "api", "docs_expand_beach_expected_output.json")) as f:
        want = json.load(f)
    got = json.loads(out[0])
    assert _canon(got) == _canon(want)
    # encoding/json field order: type, children, tuple; compact
    assert out[0].startswith('{"type":"union","children":[')
    assert '"tuple":{"namespace":"","object":"","relation":"","subject_set":{"namespace":"files"' in out[0]


def _subject_tree_class():
    """SubjectTree and friends from their field numbers (expand_service.proto:64-92,
    relation_tuples.proto:13-74), for decoding only."""
    fd = descriptor_pb2.FileDescriptorProto(name="keto_test.proto", package="kt", syntax="proto3")
    T = descriptor_pb2.FieldDescriptorProto
    def msg(name, fields, oneof=None):
        m = fd.message_type.add(name=name)
        if oneof:
            m.oneof_decl.add(name=oneof)
        for fname, num, ftype, tname, label, in_oneof in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
            if in_oneof:
                f.oneof_index = 0
    OPT, REP = T.LABEL_OPTIONAL, T.LABEL_REPEATED
    msg("SubjectSet", [("namespace", 1, T.TYPE_STRING, None, OPT, False), ("object", 2, T.TYPE_STRING, None, OPT, False),
                       ("relation", 3, T.TYPE_STRING, None, OPT, False)])
    msg("Subject", [("id", 1, T.TYPE_STRING, None, OPT, True), ("set", 2, T.TYPE_MESSAGE, ".kt.SubjectSet", OPT, True)],
        oneof="ref")
    msg("RelationTuple", [("namespace", 1, T.TYPE_STRING, None, OPT, False), ("object", 2, T.TYPE_STRING, None, OPT, False),
                          ("relation", 3, T.TYPE_STRING, None, OPT, False),
                          ("subject", 4, T.TYPE_MESSAGE, ".kt.Subject", OPT, False)])
    e = fd.enum_type.add(name="NodeType")
    for n, v in (("NODE_TYPE_UNSPECIFIED", 0), ("NODE_TYPE_UNION", 1), ("NODE_TYPE_EXCLUSION", 2),
                 ("NODE_TYPE_INTERSECTION", 3), ("NODE_TYPE_LEAF", 4)):
        e.value.add(name=n, number=v)
    msg("SubjectTree", [("node_type", 1, T.TYPE_ENUM, ".kt.NodeType", OPT, False),
                        ("subject", 2, T.TYPE_MESSAGE, ".kt.Subject", OPT, False),
                        ("tuple", 4, T.TYPE_MESSAGE, ".kt.RelationTuple", OPT, False),
                        ("children", 3, T.TYPE_MESSAGE, ".kt.SubjectTree", REP, False)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("kt.SubjectTree"))


def _proto_to_api(m):
    """SubjectTree -> the ketoapi JSON shape (TreeFromProto, ketoapi/enc_proto.go:135-165)"""
    names = {1: "union", 2: "exclusion", 3: "intersection", 4: "leaf"}
    s = m.tuple.subject
    tup = {"namespace": m.tuple.namespace, "object": m.tuple.object, "relation": m.tuple.relation}
    if s.WhichOneof("ref") == "set":
        tup["subject_set"] = {"namespace": s.set.namespace, "object": s.set.object, "relation": s.set.relation}
    else:
        tup["subject_id"] = s.id
    d = {"type": names.get(m.node_type, "unspecified"), "tuple": tup}
    if len(m.children):
        d["children"] = [_proto_to_api(c) for c in m.children]
    return d


def test_proto_decodes_to_the_same_tree_and_is_canonical():
    _, nodes, names = _beach()
    raw = api.trees_to_proto(nodes, np.array([0, len(nodes)], np.uint64), names)[0]
    cls = _subject_tree_class()
    m = cls()
    m.ParseFromString(raw)
    with open(os.path.join(GOLDEN, "api", "docs_expand_beach_expected_output.json")) as f:
        want = json.load(f)
    assert _canon(_proto_to_api(m)) == _canon(want)
    # the deprecated subject field mirrors tuple.subject on every node (enc_proto.go:125-128)
    def walk(x):
        assert x.subject == x.tuple.subject
        for c in x.children:
            walk(c)
    walk(m)
    # field-number order, defaults omitted: byte-identical to protobuf's own deterministic encoding
    assert m.SerializeToString(deterministic=True) == raw


def test_batch_nil_trees_capacity_and_escaping():
    ns, rels = ["ns<&>"], ["", "r\u2028"]
    uuids = ["plain", 'q"uote\\back\nline\x01\u2028', "\u00e9t\u00e9", b"bad\xff"]
    names = api.NameTables(ns, rels, uuids)
    T = km.TREE_DT
    a = np.array([(1, 1, 0, 0, 1, 2), (4, 0, 1, 0, 0, 0), (4, 0, 2, 0, 0, 0)], dtype=T)
    b = np.array([(4, 0, 0, 0, 0, 0)], dtype=T)
    nodes = np.concatenate([a, b])
    offs = np.array([0, 3, 3, 4], np.uint64)  # tree 1 is nil
    out = api.trees_to_json(nodes, offs, names)
    assert out[1] is None
    t0 = json.loads(out[0])
    assert t0["tuple"]["subject_set"] == {"namespace": "ns<&>", "object": "plain", "relation": "r\u2028"}
    assert [c["tuple"]["subject_id"] for c in t0["children"]] == [uuids[1], uuids[2]]
    assert "\\u003c\\u0026\\u003e" in out[0] and "\\u2028" in out[0] and "\\u0001" in out[0]
    assert json.loads(out[2]) == {"type": "leaf", "tuple": {"namespace": "", "object": "", "relation": "",
                                                            "subject_id": "plain"}}
    bad = api.trees_to_json(np.array([(4, 0, 3, 0, 0, 0)], dtype=T), np.array([0, 1], np.uint64), names)[0]
    assert json.loads(bad)["tuple"]["subject_id"] == "bad\ufffd"  # invalid UTF-8, as encoding/json does
    prot = api.trees_to_proto(nodes, offs, names)
    assert prot[1] is None and len(prot[0]) > 0 and len(prot[2]) > 0
    # malformed pre-order (a child count past the end) is rejected
    with pytest.raises(km.KetoError):
        api.trees_to_json(a[:2], np.array([0, 2], np.uint64), names)
