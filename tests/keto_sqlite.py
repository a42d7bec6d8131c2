"""Test infrastructure: write relation tuples into a SQLite file laid out like Keto's store.

The DDL below is written for these tests from the column list of
`keto_relation_tuples` / `keto_uuid_mappings` (the reference's sqlite migrations,
`...add-on-delete-cascade-to-relationship.sqlite.up.sql:14-49`,
`...uuid-mapping-remove-check.sqlite.up.sql`).  It is not the reference's migration text.
Values are written the way gobuffalo/pop + gofrs/uuid store them: UUIDs as canonical text,
strings through UUIDv5(nid, s) with a keto_uuid_mappings row each."""
import sqlite3
import uuid

import numpy as np

import refsem

DDL = """
CREATE TABLE networks (id UUID NOT NULL PRIMARY KEY, created_at TIMESTAMP, updated_at TIMESTAMP);
CREATE TABLE keto_uuid_mappings (id UUID NOT NULL PRIMARY KEY, string_representation TEXT NOT NULL);
CREATE TABLE keto_relation_tuples (
  shard_id UUID NOT NULL, nid UUID NOT NULL, namespace VARCHAR(200) NOT NULL, object UUID NOT NULL,
  relation VARCHAR(64) NOT NULL, subject_id UUID NULL, subject_set_namespace VARCHAR(200) NULL,
  subject_set_object UUID NULL, subject_set_relation VARCHAR(64) NULL, commit_time TIMESTAMP NOT NULL,
  PRIMARY KEY (shard_id, nid));
"""


def shard_uuid(order: int, rng) -> str:
    """a UUIDv4 whose text order is `order` (hand-written fixtures: insertion order is the
    shard order their expectations assume)"""
    lo = int(rng.integers(0, 2**62))
    v = (order << 80) | (0x4 << 76) | (int(rng.integers(0, 2**12)) << 64) | (0x2 << 62) | lo
    return str(uuid.UUID(int=v))


def write_store(path: str, tuples: list, nid: str = None, seed: int = 0, networks: int = 1) -> str:
    """tuples: fixture strings ('ns:obj#rel@subject').  Rows are inserted in a shuffled order;
    their shard_ids encode the fixture order.  Returns the nid."""
    rng = np.random.default_rng(seed)
    nid = uuid.UUID(nid) if nid else uuid.UUID(int=int(rng.integers(0, 2**62)) << 64 | 0x8000000000004000)
    con = sqlite3.connect(path)
    con.executescript(DDL)
    con.execute("INSERT INTO networks (id) VALUES (?)", (str(nid),))
    maps = {}

    def u(s):
        x = str(uuid.uuid5(nid, s))
        maps[x] = s
        return x

    rows = []
    for i, s in enumerate(tuples):
        t = refsem.parse_tuple(s)
        row = [shard_uuid(i, rng), str(nid), t["ns"], u(t["obj"]), t["rel"], None, None, None, None,
               f"2024-01-01 00:00:{i % 60:02d}"]
        if "subject_set" in t:
            sns, sobj, srel = t["subject_set"]
            row[6], row[7], row[8] = sns, u(sobj), srel
        else:
            row[5] = u(t["subject_id"])
        rows.append(row)
    for k in rng.permutation(len(rows)):
        con.execute("INSERT INTO keto_relation_tuples VALUES (?,?,?,?,?,?,?,?,?,?)", rows[k])
    for k in range(1, networks):  # other networks' rows must not leak in
        other = str(uuid.UUID(int=k))
        con.execute("INSERT INTO networks (id) VALUES (?)", (other,))
        for r in rows[:3]:
            con.execute("INSERT INTO keto_relation_tuples VALUES (?,?,?,?,?,?,?,?,?,?)",
                        [shard_uuid(10_000 + k, rng), other] + r[2:])
    con.executemany("INSERT OR IGNORE INTO keto_uuid_mappings VALUES (?, ?)", list(maps.items()))
    con.commit()
    con.close()
    return str(nid)


def subject_of(t: dict):
    return t["subject_set"] if "subject_set" in t else t["subject_id"]


def oracle_world(store):
    """an oracle World whose interners are the loader's (same ids as the product snapshot)"""
    w = refsem.World(namespaces=store.namespaces, strict=store.strict)
    w.ns_names, w.rel_names, w.uuids = refsem.Interner(), refsem.Interner(), refsem.Interner()
    for n in store.ns.names:
        w.ns_names(n)
    for r in store.rel.names:
        w.rel_names(r)
    for x in store.uuids.names[: store.n_uuids]:
        w.uuids(x)
    w._walk_names()
    t = store.tuples.view(refsem.TUPLE_DT).copy()  # same 48-byte record, shard bytes raw
    return w, t
