"""Transcribe the reference's own known-answer vectors into JSON fixtures.

Every vector below is copied by hand from an assertion in the reference's
tests or docs samples (file:line given per fixture / case, paths relative to
/root/reference).  Nothing here runs or imports the reference: the expected
values are the ones its tests assert.  Run `python tests/golden/make_golden.py`
to regenerate the committed JSON.

Conventions:
  * tuples are ketoapi string form `ns:obj#rel@subject` (enc_string.go:40-75);
    the reference tests assign random UUIDv4 shard ids, and none of the
    assertions depends on their order, so the fixture's list order is used;
  * namespaces use the AST JSON form of internal/schema/.snapshots
    (`{ns: [relation, ...]}`, relation = {name, types, rewrite});
  * "global" overrides limit.max_read_depth for one case (config default 5,
    embedx/config.schema.json:368-375); "depth" is the request max-depth;
  * expand trees compare child order-insensitively, as the reference's
    expand/testhelper.go:23-53 does.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def css(r):
    return {"relation": r}


def ttu(r, c):
    return {"relation": r, "computed_subject_set_relation": c}


def OR(*c):
    return {"operator": "or", "children": list(c)}


def AND(*c):
    return {"operator": "and", "children": list(c)}


def NOT(c):
    return {"inverted": c}


def leaf_id(s):
    return {"type": "leaf", "tuple": {"subject_id": s}}


def sset(ns, obj, rel):
    return {"subject_set": {"namespace": ns, "object": obj, "relation": rel}}


def leaf_set(ns, obj, rel):
    return {"type": "leaf", "tuple": sset(ns, obj, rel)}


def union(ns, obj, rel, *children):
    return {"type": "union", "tuple": sset(ns, obj, rel), "children": list(children)}


FIXTURES = {}

# ---------------------------------------------------------------------------
# internal/check/engine_test.go
FIXTURES["engine_max_depth"] = {
    "src": "internal/check/engine_test.go:82-126",
    "namespaces": {"test": []},
    "tuples": ["test:object#admin@user", "test:object#owner@test:object#admin",
               "test:object#access@test:object#owner"],
    "checks": [
        {"query": "test:object#access@user", "depth": 2, "allowed": False, "src": ":103-106"},
        {"query": "test:object#access@user", "depth": 3, "allowed": True, "src": ":108-111"},
        {"query": "test:object#access@user", "depth": 2, "global": 2, "allowed": False, "src": ":113-117"},
        {"query": "test:object#access@user", "depth": 0, "global": 3, "allowed": True, "src": ":119-123"},
    ],
}
FIXTURES["engine_direct_inclusion"] = {
    "src": "internal/check/engine_test.go:128-160",
    "namespaces": {"n": [], "u": []},
    "tuples": ["n:o#r@subject_id", "n:o#r@u:with_relation#r", "n:o#r@u:empty_relation#",
               "n:o#r@u:missing_relation"],
    "checks": [{"query": q, "depth": 0, "allowed": True, "src": ":141-149"} for q in [
        "n:o#r@subject_id", "n:o#r@u:with_relation#r", "n:o#r@u:empty_relation",
        "n:o#r@u:empty_relation#", "n:o#r@u:missing_relation", "n:o#r@u:missing_relation#"]],
}
FIXTURES["engine_indirect_level1"] = {
    "src": "internal/check/engine_test.go:162-199",
    "namespaces": {"sofa": []},
    "tuples": ["sofa:dust#have to remove@sofa:dust#producer", "sofa:dust#producer@mark"],
    "checks": [{"query": "sofa:dust#have to remove@mark", "depth": 0, "allowed": True, "src": ":189-198"}],
}
FIXTURES["engine_direct_exclusion"] = {
    "src": "internal/check/engine_test.go:201-223",
    "namespaces": {"TestEngine/direct_exclusion": []},
    "tuples": ["TestEngine/direct_exclusion:obj#relation@user"],
    "checks": [{"query": "TestEngine/direct_exclusion:obj#relation@other_user", "depth": 0,
                "allowed": False, "src": ":214-222"}],
}
FIXTURES["engine_subject_expansion"] = {
    "src": "internal/check/engine_test.go:225-267",
    "namespaces": {"n": [{"name": "r", "types": [{"namespace": "n", "relation": "r"}]}]},
    "tuples": ["n:a#r@n:b#r", "n:b#r@n:c#r", "n:c#r@n:d#r", "n:d#r@u"],
    "checks": [{"query": q, "depth": 0, "allowed": True, "src": ":251-265"} for q in [
        "n:d#r@u", "n:c#r@u", "n:b#r@u", "n:a#r@u"]],
}
FIXTURES["engine_wrong_object"] = {
    "src": "internal/check/engine_test.go:269-298",
    "namespaces": {"": []},
    "tuples": [":object#access@:object#owner", ":other_object#owner@user"],
    "checks": [{"query": ":object#access@user", "depth": 0, "allowed": False, "src": ":290-297"}],
}
FIXTURES["engine_wrong_relation"] = {
    "src": "internal/check/engine_test.go:300-335",
    "namespaces": {"diaries": []},
    "tuples": ["diaries:entry#read@diaries:entry#author", "diaries:entry#not author@user"],
    "checks": [{"query": "diaries:entry#read@user", "depth": 0, "allowed": False, "src": ":327-334"}],
}
FIXTURES["engine_indirect_level2"] = {
    "src": "internal/check/engine_test.go:337-360",
    "namespaces": {"obj": [], "org": []},
    "tuples": ["obj:object#write@obj:object#owner", "obj:object#owner@org:organization#member",
               "org:organization#member@user"],
    "checks": [
        {"query": "obj:object#write@user", "depth": 0, "allowed": True, "src": ":350-353"},
        {"query": "org:organization#member@user", "depth": 0, "allowed": True, "src": ":355-358"},
    ],
}
FIXTURES["engine_rejects_transitive"] = {
    "src": "internal/check/engine_test.go:362-395",
    "namespaces": {"2": []},
    "tuples": [":file#parent@:directory#", ":directory#access@user"],
    "checks": [{"query": ":file#access@user", "depth": 0, "allowed": False, "src": ":387-394"}],
}
FIXTURES["engine_subject_id_next_to_set"] = {
    "src": "internal/check/engine_test.go:397-445",
    "namespaces": {"39231": []},
    "tuples": ["39231:obj#owner@directOwner", "39231:obj#owner@39231:org#member",
               "39231:org#member@indirectOwner"],
    "checks": [
        {"query": "39231:obj#owner@directOwner", "depth": 0, "allowed": True, "src": ":426-434"},
        {"query": "39231:obj#owner@indirectOwner", "depth": 0, "allowed": True, "src": ":436-444"},
    ],
}
FIXTURES["engine_wide_graph"] = {
    "src": "internal/check/engine_test.go:447-482",
    "namespaces": {"9234": []},
    "tuples": ["9234:obj#access@9234:org0#member", "9234:obj#access@9234:org1#member",
               "9234:org0#member@user0", "9234:org1#member@user1", "9234:org0#member@user2",
               "9234:org1#member@user3"],
    "checks": [{"query": f"9234:obj#access@user{i}", "depth": 0, "allowed": True, "src": ":470-481"}
               for i in range(4)],
}
FIXTURES["engine_circular"] = {
    "src": "internal/check/engine_test.go:484-548",
    "namespaces": {"7743": []},
    "tuples": ["7743:Sendlinger Tor#connected@7743:Odeonsplatz#connected",
               "7743:Odeonsplatz#connected@7743:Central Station#connected",
               "7743:Central Station#connected@7743:Sendlinger Tor#connected"],
    "checks": [{"query": "7743:Sendlinger Tor#connected@Central Station", "depth": 0, "allowed": False,
                "src": ":536-547"}],
}

# internal/check/testfixtures/project_opl.ts as AST (parser.go left-deep build + simplifyExpression)
PROJECT_OPL = {
    "User": [],
    "Project": [
        {"name": "owner", "types": [{"namespace": "User"}]},
        {"name": "developer", "types": [{"namespace": "User"}]},
        {"name": "isOwner", "rewrite": OR(css("owner"))},
        {"name": "isOwnerOrDeveloper", "rewrite": OR(css("owner"), css("developer"))},
        {"name": "writeCollaborator", "rewrite": OR(css("isOwner"))},
        {"name": "readCollaborator", "rewrite": OR(css("isOwnerOrDeveloper"))},
        {"name": "deleteProject", "rewrite": OR(css("isOwner"))},
        {"name": "writeProject", "rewrite": OR(css("isOwnerOrDeveloper"))},
        {"name": "readProject", "rewrite": OR(css("isOwnerOrDeveloper"))},
    ],
}
FIXTURES["engine_strict_mode"] = {
    "src": "internal/check/engine_test.go:550-578 (+ testfixtures/project_opl.ts)",
    "namespaces": PROJECT_OPL,
    "strict": True,
    "tuples": ["Project:abc#owner@User:1", "Project:abc#owner@User1", "Project:abc#isOwner@User:isOwner",
               "Project:abc#readProject@readProjectUser", "Project:abc#readProject@User:ReadProject"],
    "checks": [{"query": "Project:abc#readProject@" + s, "depth": 10, "allowed": False, "src": ":565-570"}
               for s in ["readProjectUser", "User:ReadProject", "User:isOwner"]] +
              [{"query": "Project:abc#readProject@" + s, "depth": 10, "allowed": True, "src": ":572-576"}
               for s in ["User:1", "User1"]],
}

# ---------------------------------------------------------------------------
# internal/check/rewrites_test.go
REWRITE_NS = {
    "doc": [
        {"name": "owner"},
        {"name": "editor", "rewrite": OR(css("owner"))},
        {"name": "viewer", "rewrite": OR(css("editor"), ttu("parent", "viewer"))},
    ],
    "users": [],
    "group": [{"name": "member"}],
    "level": [{"name": "member"}],
    "resource": [
        {"name": "level"},
        {"name": "viewer", "rewrite": OR(ttu("owner", "member"))},
        {"name": "owner", "rewrite": OR(ttu("owner", "member"))},
        {"name": "read", "rewrite": OR(css("viewer"), css("owner"))},
        {"name": "update", "rewrite": OR(css("owner"))},
        {"name": "delete", "rewrite": AND(css("owner"), ttu("level", "member"))},
    ],
    "acl": [
        {"name": "allow"},
        {"name": "deny"},
        {"name": "access", "rewrite": AND(css("allow"), NOT(css("deny")))},
    ],
}
_rw_cases = [
    ("doc:document#owner@users:user", True), ("doc:document#editor@users:user", True),
    ("doc:document#editor@plain_user", True), ("doc:document#viewer@users:user", True),
    ("doc:document#editor@nobody", False), ("doc:folder#viewer@users:user", True),
    ("doc:doc_in_folder#viewer@users:user", True), ("doc:doc_in_folder#viewer@plain_user", True),
    ("doc:doc_in_folder#viewer@nobody", False), ("doc:another_doc#viewer@user", False),
    ("doc:file#viewer@user", True), ("level:superadmin#member@mark", True),
    ("resource:topsecret#owner@mark", True), ("resource:topsecret#delete@mark", True),
    ("resource:topsecret#update@mike", True), ("level:superadmin#member@mike", False),
    ("resource:topsecret#delete@mike", False), ("resource:topsecret#delete@sandy", False),
    ("acl:document#access@alice", True), ("acl:document#access@bob", True),
    ("acl:document#allow@mallory", True), ("acl:document#access@mallory", False),
]
FIXTURES["rewrites"] = {
    "src": "internal/check/rewrites_test.go:23-90,109-223",
    "namespaces": REWRITE_NS,
    "tuples": [
        "doc:document#owner@plain_user", "doc:document#owner@users:user", "doc:doc_in_folder#parent@doc:folder",
        "doc:folder#owner@plain_user", "doc:folder#owner@users:user", "doc:file#parent@doc:folder_c",
        "doc:folder_c#parent@doc:folder_b", "doc:folder_b#parent@doc:folder_a", "doc:folder_a#owner@user",
        "group:editors#member@mark", "level:superadmin#member@mark", "level:superadmin#member@sandy",
        "resource:topsecret#owner@group:editors#", "resource:topsecret#level@level:superadmin#",
        "resource:topsecret#owner@mike", "acl:document#allow@alice", "acl:document#allow@bob",
        "acl:document#allow@mallory", "acl:document#deny@mallory",
    ],
    "checks": [{"query": q, "depth": 100, "allowed": a, "src": ":136-223"} for q, a in _rw_cases] +
              [{"query": "doc:file#viewer@user", "depth": 100, "allowed": True, "src": ":240-264 (one worker)"}],
}

# ---------------------------------------------------------------------------
# internal/check/bench_test.go (expected IsMember asserted inside the benchmarks)
_deep_tuples = ["deep:deep_file#parent@deep:folder_1#..."] + \
    [f"deep:folder_{i}#parent@deep:folder_{i + 1}#..." for i in range(1, 32)] + \
    [f"deep:folder_{d}#owner@user_{d}" for d in [2, 4, 8, 16, 32]] + \
    [f"{w}-wide:wide_file#editor@user" for w in [10, 20, 40, 80, 100]]
_wide_ns = {}
for _w in [10, 20, 40, 80, 100]:
    _wide_ns[f"{_w}_wide"] = [{"name": "editor"}] + [{"name": f"relation-{i}"} for i in range(_w)] + [
        {"name": "viewer", "rewrite": OR(*([css(f"relation-{i}") for i in range(_w)] + [css("editor")]))}]
FIXTURES["bench_check_engine"] = {
    "src": "internal/check/bench_test.go:56-133 (namespaces appended after registry build are not "
           "configured, :83 vs :96; tuples use the '%d-wide' namespace, :97)",
    "namespaces": {"deep": [
        {"name": "owner"},
        {"name": "editor", "rewrite": OR(css("owner"))},
        {"name": "viewer", "rewrite": OR(css("editor"), ttu("parent", "viewer"))}]},
    "global": 3200,
    "tuples": _deep_tuples,
    "checks": [{"query": f"deep:deep_file#viewer@user_{d}", "depth": 2 * d, "allowed": True, "src": ":104-116"}
               for d in [2, 4, 8, 16, 32]] +
              [{"query": f"{w}-wide:wide_file#editor@user", "depth": 2 * w, "allowed": True, "src": ":119-131"}
               for w in [10, 20, 40, 80, 100]],
    "unused_namespaces": list(_wide_ns),
}
FIXTURES["bench_computed_usersets"] = {
    "src": "internal/check/bench_test.go:138-174",
    "namespaces": PROJECT_OPL,
    "strict": True,
    "tuples": ["Project:Ory#owner@User:Admin", "Project:Ory#developer@User:Dev"],
    "checks": [{"query": "Project:Ory#readProject@User:Dev", "depth": 0, "allowed": True, "src": ":160-170"}],
}

# ---------------------------------------------------------------------------
# internal/e2e/testcases_test.go (engine-visible parts)
FIXTURES["e2e_cases"] = {
    "src": "internal/e2e/testcases_test.go:47-163",
    "namespaces": {"creates": [], "empty": [], "selfset": [], "expand": []},
    "tuples": ["creates:object for client#access@client", "empty:#access@", "empty:#access@empty:#access",
               "selfset:obj for client#check@selfset:obj for client#check",
               "expand:tree for client#expand@s1", "expand:tree for client#expand@s2"],
    "checks": [
        {"query": "creates:object for client#access@client", "depth": 0, "allowed": True, "src": ":56-74"},
        {"query": "empty:#access@", "depth": 0, "allowed": True, "src": ":76-101"},
        {"query": "empty:#access@empty:#access", "depth": 0, "allowed": True, "src": ":76-101"},
        {"query": "selfset:obj for client#check@selfset:obj for client#check", "depth": 0, "allowed": True,
         "src": ":103-122"},
    ],
    "expands": [{"subject": "expand:tree for client#expand", "depth": 100, "src": ":124-163",
                 "tree": union("expand", "tree for client", "expand", leaf_id("s1"), leaf_id("s2"))}],
}

# ---------------------------------------------------------------------------
# internal/expand/engine_test.go
FIXTURES["expand_engine"] = {
    "src": "internal/expand/engine_test.go:58-393",
    "namespaces": {"": [], "92384": []},
    "tuples": [
        ":boulder_group#member@tommy", ":boulder_group#member@paul",
        ":root_t#transitive member@:g1#member", ":g1#member@u11", ":g1#member@u12", ":g1#member@u13",
        ":root_t#transitive member@:g2#member", ":g2#member@u21", ":g2#member@u22", ":g2#member@u23",
        ":id0#child@:id1#child", ":id1#child@:id2#child", ":id2#child@:id3#child", ":id3#child@:id4#child",
        ":root_p#access@pu0", ":root_p#access@pu1", ":root_p#access@pu2", ":root_p#access@pu3",
        ":leaf_root#rel@:leaf_obj#sr",
        "92384:Sendlinger Tor#connected@92384:Odeonsplatz#connected",
        "92384:Odeonsplatz#connected@92384:Central Station#connected",
        "92384:Central Station#connected@92384:Sendlinger Tor#connected",
    ],
    "expands": [
        {"subject_id": "some_user", "depth": 100, "src": ":59-69", "tree": leaf_id("some_user")},
        {"subject": ":boulder_group#member", "depth": 100, "src": ":71-109",
         "tree": union("", "boulder_group", "member", leaf_id("paul"), leaf_id("tommy"))},
        {"subject": ":root_t#transitive member", "depth": 100, "src": ":111-188",
         "tree": union("", "root_t", "transitive member",
                       union("", "g1", "member", leaf_id("u11"), leaf_id("u12"), leaf_id("u13")),
                       union("", "g2", "member", leaf_id("u21"), leaf_id("u22"), leaf_id("u23")))},
        {"subject": ":id0#child", "depth": 4, "src": ":190-246", "exact": True,
         "tree": union("", "id0", "child", union("", "id1", "child", union("", "id2", "child",
                                                                            leaf_set("", "id3", "child"))))},
        {"subject": ":root_p#access", "depth": 10, "src": ":248-278",
         "tree": union("", "root_p", "access", *[leaf_id(f"pu{i}") for i in range(4)])},
        {"subject": ":leaf_root#rel", "depth": 100, "src": ":280-309", "exact": True,
         "tree": union("", "leaf_root", "rel", leaf_set("", "leaf_obj", "sr"))},
        {"subject": "92384:Sendlinger Tor#connected", "depth": 100, "src": ":311-382", "exact": True,
         "tree": union("92384", "Sendlinger Tor", "connected",
                       union("92384", "Odeonsplatz", "connected",
                             union("92384", "Central Station", "connected",
                                   leaf_set("92384", "Sendlinger Tor", "connected"))))},
        {"subject": "unknown:obj#rel", "depth": 100, "src": ":384-393", "tree": None},
    ],
}

# ---------------------------------------------------------------------------
# contrib/docs-code-samples
FIXTURES["docs_expand_beach"] = {
    "src": "contrib/docs-code-samples/expand-api-display-access/{00-create-tuples/cli.sh,"
           "01-expand-beach/cli.sh,01-expand-beach/expected_output.json,keto.yml}",
    "namespaces": {"files": [], "directories": []},
    "tuples": ["directories:/photos#owner@maureen", "files:/photos/beach.jpg#owner@maureen",
               "files:/photos/mountains.jpg#owner@laura", "directories:/photos#access@laura",
               "directories:/photos#access@(directories:/photos#owner)",
               "files:/photos/beach.jpg#access@(files:/photos/beach.jpg#owner)",
               "files:/photos/beach.jpg#access@(directories:/photos#access)",
               "files:/photos/mountains.jpg#access@(files:/photos/mountains.jpg#owner)",
               "files:/photos/mountains.jpg#access@(directories:/photos#access)"],
    "expands": [{"subject": "files:/photos/beach.jpg#access", "depth": 3, "src": "expected_output.json",
                 "tree": union("files", "/photos/beach.jpg", "access",
                               union("files", "/photos/beach.jpg", "owner", leaf_id("maureen")),
                               union("directories", "/photos", "access", leaf_id("laura"),
                                     leaf_set("directories", "/photos", "owner")))}],
}
FIXTURES["docs_simple_check"] = {
    "src": "contrib/docs-code-samples/simple-access-check-guide/{00-write-direct-access,01-check-direct-access}",
    "namespaces": {"messages": []},
    "tuples": ["messages:02y_15_4w350m3#decypher@john"],
    "checks": [{"query": "messages:02y_15_4w350m3#decypher@john", "depth": 0, "allowed": True,
                "src": "01-check-direct-access/expected_output.txt: Allowed"}],
}

# ---------------------------------------------------------------------------
# contrib/cat-videos-example (BASELINE config 1 plumbing); answers derived by
# hand from the 7 tuples (no reference assertion exists for these queries).
FIXTURES["cat_videos"] = {
    "src": "contrib/cat-videos-example/{keto.yml,relation-tuples/*.json} (answers hand-derived, not "
           "asserted by the reference)",
    "derived": True,
    "namespaces": {"videos": []},
    "tuples": ["videos:/cats/1.mp4#owner@videos:/cats#owner", "videos:/cats/1.mp4#view@videos:/cats/1.mp4#owner",
               "videos:/cats/1.mp4#view@*", "videos:/cats/2.mp4#owner@videos:/cats#owner",
               "videos:/cats/2.mp4#view@videos:/cats/2.mp4#owner", "videos:/cats#owner@cat lady",
               "videos:/cats#view@videos:/cats#owner"],
    "checks": [
        {"query": "videos:/cats/1.mp4#view@*", "depth": 0, "allowed": True},
        {"query": "videos:/cats/2.mp4#view@*", "depth": 0, "allowed": False},
        {"query": "videos:/cats/1.mp4#view@cat lady", "depth": 0, "allowed": True},
        {"query": "videos:/cats/2.mp4#owner@cat lady", "depth": 0, "allowed": True},
        {"query": "videos:/cats#view@cat lady", "depth": 0, "allowed": True},
        {"query": "videos:/cats/2.mp4#view@nobody", "depth": 0, "allowed": False},
        {"query": "videos:/cats/1.mp4#view@cat lady", "depth": 2, "allowed": False},
    ],
}

# ---------------------------------------------------------------------------
# Hand-derived cases for two reference behaviours no reference test pins (answers derived
# from the reference source, cited per case; "derived": True marks them as such).

# H3: the visited key is UUIDv5(obj, ns+"-"+rel) (relationtuple/definitions.go:114-116,
# x/graph/graph_utils.go:45-53), so a-b:o#c and a:o#b-c are ONE visited node.  Fixture order
# is shard order.  root#m's row is [a-b:o#c, a:o#b-c]; the found-lookahead (traverser.go:73-80)
# finds alice directly in neither; the child loop (engine.go:151-162) visits a-b:o#c (nothing
# below it) and then skips a:o#b-c as already visited, so alice -- reachable only through
# a:o#b-c -> g:x#m -- is NOT found.  bob, in a-b:o#c's own subtree, is.  Expand (global visited
# set incl. the root, expand/engine.go:69-72) shows the second set as a leaf.
FIXTURES["visited_alias_h3"] = {
    "src": "relationtuple/definitions.go:114-116 + x/graph/graph_utils.go:45-53 (hand-derived)",
    "derived": True,
    "namespaces": {"g": [], "a-b": [], "a": []},
    "tuples": ["g:root#m@(a-b:o#c)", "g:root#m@(a:o#b-c)", "a-b:o#c@(g:y#m)", "g:y#m@bob",
               "a:o#b-c@(g:x#m)", "g:x#m@alice", "g:other#m@(a:o#b-c)"],
    "checks": [
        {"query": "g:root#m@alice", "depth": 0, "allowed": False, "src": "alias prunes a:o#b-c"},
        {"query": "g:root#m@bob", "depth": 0, "allowed": True, "src": "a-b:o#c -> g:y#m"},
        {"query": "g:other#m@alice", "depth": 0, "allowed": True, "src": "no collision in this scope"},
        {"query": "a:o#b-c@alice", "depth": 0, "allowed": True, "src": "root not inserted (engine.go:119)"},
    ],
    "expands": [
        {"subject": "g:root#m", "depth": 5, "src": "expand/engine.go:69-72, 106-119", "exact": True,
         "tree": union("g", "root", "m", union("a-b", "o", "c", union("g", "y", "m", leaf_id("bob"))),
                       leaf_set("a", "o", "b-c"))},
    ],
}

# Sibling marking order (engine.go:151-162 + concurrent_checkgroup.go:150-159): g.Add(check_A)
# returns as soon as check_A is handed to the consumer, so the loop marks B before A's subtree
# makes its first read.  root#view = [A#member, B#member], A#member includes B#member, alice is
# in C#member below B.  Global depth 3: ES(root#view, 2) -> A at 2: A's ES (1) sees B already
# visited and skips it; B at 2: ES(B, 1) finds alice in C#member by lookahead -> allowed.  (If
# A's subtree ran before B was marked, A would reach B at depth 1, miss, and B would then be
# skipped: denied.)  Depth 2: B's ES would run at 0 -> Unknown -> denied.  Depth 4: allowed.
FIXTURES["sibling_marking_order"] = {
    "src": "internal/check/engine.go:151-162, checkgroup/concurrent_checkgroup.go:150-159 (hand-derived)",
    "derived": True,
    "namespaces": {"g": []},
    "tuples": ["g:root#view@(g:A#member)", "g:root#view@(g:B#member)", "g:A#member@(g:B#member)",
               "g:B#member@(g:C#member)", "g:C#member@alice"],
    "checks": [
        {"query": "g:root#view@alice", "depth": 3, "allowed": True, "src": "B marked before A runs"},
        {"query": "g:root#view@alice", "depth": 2, "allowed": False, "src": "depth ledger"},
        {"query": "g:root#view@alice", "depth": 4, "allowed": True, "src": "both orders"},
        {"query": "g:A#member@alice", "depth": 3, "allowed": True, "src": "A -> B -> C by lookahead"},
    ],
}


def main():
    for name, fx in FIXTURES.items():
        fx = dict(fx)
        fx["name"] = name
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
            f.write("\n")
    print(f"wrote {len(FIXTURES)} fixtures to {HERE}")


if __name__ == "__main__":
    main()
