"""TEST INFRASTRUCTURE ONLY -- the reference's Check engine under its real concurrency.

refsem.c evaluates a check as a recursion in one canonical schedule (SCHED_EAGER) plus the
sequential one.  The reference runs it as goroutines (internal/check/engine.go,
rewrites.go, binop.go, checkgroup/concurrent_checkgroup.go), and the visited set
(x/graph/graph_utils.go:38-53) is shared by every goroutine below the expand-subject that
created it, so which occurrence of a subject set gets explored depends on timing.  This module
restates that engine at goroutine granularity and runs it under a seeded scheduler, so a test
can ask: does any legal interleaving change a query's answer?

What is modelled, each with the reference line it follows:
  - goroutines are Python generators; a blocking operation yields a readiness predicate and a
    hop (an SQL statement, a visited mark) yields None.  The scheduler advances one ready
    goroutine per step, chosen by the policy ("random", "newest", "oldest") from a seed;
  - contexts carry the visited set as a value and cancel their descendants
    (context.WithCancel; graph.InitVisited / CheckAndAddVisited, graph_utils.go:38-53);
  - concurrentCheckgroup (concurrent_checkgroup.go:66-138): one reservation, so a group runs
    its checks one after another, but Add returns once the check is handed to the consumer
    (:150-159); the first Err / IsMember wins, the group's sub-context is cancelled when the
    consumer returns (:72), Result / CheckFunc finalize (:170-200);
  - construction is eager, as in Go: checkIsAllowed (engine.go:214-249) creates its group and
    Adds its sub-checks while it is being built -- so building child k+1 of an expand-subject
    (engine.go:161, the argument of g.Add) already starts k+1's first sub-check while child k
    runs, and blocks until that sub-check finishes if k+1 has another;
    checkSubjectSetRewrite (rewrites.go:33-134) builds its computed-subject-set, nested
    rewrite and NOT children when it is built, checkInverted (rewrites.go:136-200) its child;
  - or / and (binop.go:18-73) call each check synchronously in the rewrite's goroutine and
    read the results in order;
  - a goroutine whose context was cancelled fails its next SQL statement (the driver's
    context check) but keeps running what needs no statement -- an expand-subject loop keeps
    marking its remaining siblings (engine.go:151-162).

Not modelled: GetRelationTuples paging (one page; the worlds here hold fewer rows than a page),
the SQL statements' own latency (any is covered by the scheduler's choices), Go's select
picking between a result and a cancellation in a group whose answer is already decided (only
cancelled sub-trees see it, and their answers are never read).
"""
from __future__ import annotations

import numpy as np

import refsem

IS, NOT, UNK = refsem.IS_MEMBER, refsem.NOT_MEMBER, refsem.UNKNOWN
ERR_NO_RELATION, ERR_NOT_IMPLEMENTED, ERR_CANCELED = 1, 3, 100


def decisive(r):
    return r[1] != 0 or r[0] == IS


class Deadlock(RuntimeError):
    pass


class ReferenceCrash(RuntimeError):
    """building the check recursed without end: an AND's computed subject set (or a NOT's)
    that reaches its own relation again keeps restDepth (rewrites.go:208-230), so the
    reference's construction never returns (the goroutine's stack overflows).  Such a query
    has no reference answer; refsem.c stops it at MAX_RECURSION with an internal error."""


MAX_NEST = 300


class _Task:
    __slots__ = ("gen", "wait", "seq")

    def __init__(self, gen, seq):
        self.gen, self.wait, self.seq = gen, None, seq


class Sched:
    """cooperative goroutine scheduler: a ready goroutine runs until its next yield"""

    def __init__(self, rng: np.random.Generator, policy: str = "random"):
        self.rng, self.policy = rng, policy
        self.tasks: list[_Task] = []
        self.seq = 0
        self.steps = 0

    def go(self, gen):
        self.seq += 1
        self.tasks.append(_Task(gen, self.seq))

    def coin(self) -> bool:
        return bool(self.rng.integers(0, 2))

    def run_until(self, done, max_steps=5_000_000):
        while not done():
            ready = [t for t in self.tasks if t.wait is None or t.wait()]
            if not ready:
                raise Deadlock("no goroutine can run and the check has no answer")
            if self.policy == "newest":
                t = max(ready, key=lambda x: x.seq) if self.rng.random() < 0.9 else ready[self.rng.integers(len(ready))]
            elif self.policy == "oldest":
                t = min(ready, key=lambda x: x.seq) if self.rng.random() < 0.9 else ready[self.rng.integers(len(ready))]
            else:
                t = ready[self.rng.integers(len(ready))]
            try:
                t.wait = t.gen.send(None)
            except StopIteration:
                self.tasks.remove(t)
            self.steps += 1
            if self.steps > max_steps:
                raise RuntimeError("simulation step limit")


class Future:
    __slots__ = ("done", "value")

    def __init__(self):
        self.done, self.value = False, None

    def set(self, v):
        if not self.done:
            self.done, self.value = True, v


class Ctx:
    """context.Context: a visited set as value, cancellation flowing to descendants"""

    def __init__(self, parent=None, visited=None):
        self.parent = parent
        self.visited = visited if visited is not None else (parent.visited if parent else None)
        self.cancelled = parent.cancelled if parent else False
        self.children: list[Ctx] = []
        self.on_cancel = []
        if parent is not None and not self.cancelled:
            parent.children.append(self)

    def cancel(self):
        if self.cancelled:
            return
        self.cancelled = True
        for cb in self.on_cancel:
            cb()
        for c in self.children:
            c.cancel()


class Group:
    """concurrentCheckgroup (checkgroup/concurrent_checkgroup.go:49-200); the consumer
    goroutine's state transitions run when the event that triggers them happens"""

    def __init__(self, e: "Engine", ctx: Ctx):
        self.e, self.ctx = e, ctx
        self.sub = Ctx(ctx)  # context.WithCancel(g.ctx) (:58)
        self.total = self.finished = 0
        self.finalizing = self.done = False
        self.result = (UNK, 0)
        self.reserve = True  # "Start with one reservation available." (:89)
        self.sub.on_cancel.append(self._sub_done)
        if self.sub.cancelled:
            self._sub_done()

    def _finish(self, r):  # return from the consumer: result set, doneCh closed, cancel (:72-75)
        if not self.done:
            self.done, self.result = True, r
            self.sub.cancel()

    def _sub_done(self):  # case <-g.subcheckCtx.Done() (:127-129)
        self._finish((UNK, ERR_CANCELED if self.ctx.cancelled else 0))

    def deliver(self, r):  # case result := <-resultCh (:112-124)
        if self.done:
            return  # receiveRemaining
        self.finished += 1
        if decisive(r):
            self._finish(r)
        elif self.finalizing and self.finished == self.total:
            self._finish((NOT, 0))
        else:
            self.reserve = True

    def add(self, check):
        """Add (:150-159): take the reservation (or see the sub-context done), hand the check
        to the consumer, which starts it as a goroutine unless it is finalizing (:93-98)"""
        yield lambda: self.reserve or self.sub.cancelled
        if self.sub.cancelled and (not self.reserve or self.e.sched.coin()):
            return
        self.reserve = False
        if self.done or self.finalizing:
            return
        self.total += 1
        self.e.sched.go(check(self.sub, self.deliver))

    def try_finalize(self):  # (:176-181, :99-111)
        if self.done or self.finalizing:
            return
        self.finalizing = True
        if self.finished == self.total:
            self._finish((NOT, 0))

    def wait_result(self):  # Result (:184-188)
        self.try_finalize()
        yield lambda: self.done
        return self.result

    def check_func(self):  # CheckFunc (:191-202)
        def f(ctx, send):
            self.try_finalize()
            yield lambda: self.done or ctx.cancelled
            if not self.done:
                self.sub.cancel()
            send(self.result)
        return f


def _const(r):
    def f(ctx, send):
        send(r)
        return
        yield  # a generator function
    return f


IS_F, NOT_F, UNK_F = _const((IS, 0)), _const((NOT, 0)), _const((UNK, 0))
NOT_IMPL_F = _const((UNK, ERR_NOT_IMPLEMENTED))


class Engine:
    """the reference engine over one world, one query at a time"""

    def __init__(self, world: refsem.World, tuples: np.ndarray, shard_bytes: bool = False,
                 max_depth: int | None = None, max_width: int | None = None):
        self.w = world
        nsarr, rels, ast, children = world.flatten()
        self.vcls = world.vclass()
        self.ns_cfg = nsarr
        self.rels, self.ast, self.children = rels, ast, children
        self.empty_rel = world.rel_names.ids[""]
        self.strict = bool(world.strict)
        self.max_depth = world.max_depth if max_depth is None else max_depth
        self.max_width = world.max_width if max_width is None else max_width
        t = np.asarray(tuples).view(refsem.TUPLE_DT)
        hi, lo = t["shard_hi"].astype(np.uint64), t["shard_lo"].astype(np.uint64)
        if shard_bytes:
            hi, lo = hi.byteswap(), lo.byteswap()
        order = np.lexsort((np.arange(len(t)), lo, hi))  # ORDER BY shard_id (traverser.go:88)
        self.rows: dict = {}
        self.ex: set = set()
        for i in order:
            r = t[i]
            ns, obj, rel, kind, sid = int(r["ns"]), int(r["obj"]), int(r["rel"]), int(r["kind"]), int(r["sid"])
            sns, srel = (int(r["sns"]), int(r["srel"])) if kind == 1 else (0, 0)
            self.rows.setdefault((ns, obj, rel), []).append((kind, sid, sns, srel))
            self.ex.add((ns, obj, rel, kind, sid, sns, srel))
        self.sched: Sched | None = None
        self.subj = None

    # -- the store (persistence/sql) -------------------------------------------------------
    def _exists(self, ns, obj, rel):  # ExistsRelationTuples (relationtuples.go:249-261)
        return (ns, obj, rel) + self.subj in self.ex

    def _vkey(self, sns, sid, srel):  # SubjectSet.UniqueID (relationtuple/definitions.go:114-116)
        if sns >= self.vcls.shape[0] or srel >= self.vcls.shape[1]:
            return (sid, "x", sns, srel)
        return (sid, int(self.vcls[sns, srel]))

    def _relation_for(self, ns, rel):  # namespace.ASTRelationFor (namespace/definitions.go:37-62)
        if rel == self.empty_rel or ns >= len(self.ns_cfg) or not self.ns_cfg[ns]["configured"]:
            return -1, 0
        b, c = int(self.ns_cfg[ns]["rel_begin"]), int(self.ns_cfg[ns]["rel_count"])
        if c == 0:
            return -1, 0
        for i in range(b, b + c):
            if int(self.rels[i]["name"]) == rel:
                return i, 0
        return -1, ERR_NO_RELATION

    # -- engine.go -------------------------------------------------------------------------
    def check_is_allowed(self, ctx, ns, obj, rel, d, skip_direct, nest=0):
        """checkIsAllowed (engine.go:214-249): builds the group and Adds while being built"""
        if d <= 0:
            return UNK_F
        if nest > MAX_NEST:
            raise ReferenceCrash()
        g = Group(self, ctx)
        ri, err = self._relation_for(ns, rel)
        if err:
            yield from g.add(_const((UNK, err)))
            return g.check_func()
        has_rw = ri >= 0 and int(self.rels[ri]["rewrite"]) >= 0
        can_ss = not self.strict or ri < 0 or bool(self.rels[ri]["has_ss_type"])
        if has_rw:
            cf = yield from self.check_rewrite(ctx, ns, obj, int(self.rels[ri]["rewrite"]), d, nest + 1)
            yield from g.add(cf)
        if (not self.strict or not has_rw) and not skip_direct:
            yield from g.add(self.check_direct(ns, obj, rel, d - 1))
        if can_ss:
            yield from g.add(self.check_expand_subject(ns, obj, rel, d - 1))
        return g.check_func()

    def check_direct(self, ns, obj, rel, d):  # checkDirect (engine.go:167-208)
        if d <= 0:
            return UNK_F

        def f(ctx, send):
            yield None
            if ctx.cancelled:  # the statement fails: logged, NotMember (:181-189)
                send((NOT, 0))
                return
            send((IS, 0) if self._exists(ns, obj, rel) else (NOT, 0))
        return f

    def check_expand_subject(self, ns, obj, rel, d):
        """checkExpandSubject (engine.go:102-164) + TraverseSubjectSetExpansion
        (traverser.go:53-121)"""
        if d <= 0:
            return UNK_F

        def f(ctx, send):
            g = Group(self, ctx)
            inner = ctx if ctx.visited is not None else Ctx(ctx, visited=set())  # InitVisited
            yield None  # the statement
            if ctx.cancelled:
                yield from g.add(_const((UNK, ERR_CANCELED)))
                send((yield from g.wait_result()))
                return
            results, found = [], False
            for (kind, sid, sns, srel) in self.rows.get((ns, obj, rel), ()):
                if kind != 1:
                    continue
                results.append((sns, sid, srel))
                if self._exists(sns, sid, srel):
                    found = True
                    break
            if found:
                yield from g.add(IS_F)
                send((yield from g.wait_result()))
                return
            if len(results) > self.max_width:
                results = results[: self.max_width - 1]
            for (sns, sid, srel) in results:
                yield None
                key = self._vkey(sns, sid, srel)
                if key in inner.visited:
                    continue
                inner.visited.add(key)
                cf = yield from self.check_is_allowed(inner, sns, sid, srel, d, True)
                yield from g.add(cf)
            send((yield from g.wait_result()))
        return f

    # -- rewrites.go -----------------------------------------------------------------------
    def check_rewrite(self, ctx, ns, obj, ai, d, nest=0):
        """checkSubjectSetRewrite (rewrites.go:33-134): its children are built here"""
        if d <= 0:
            return UNK_F
        a = self.ast[ai]
        op = int(a["op"])
        if op not in (0, 1):
            return NOT_IMPL_F
        kids = [int(self.children[int(a["child_begin"]) + k]) for k in range(int(a["child_count"]))]
        checks = []
        handled = set()
        if op == 0:
            css = []
            for k, ci in enumerate(kids):
                if int(self.ast[ci]["type"]) == refsem.CSS:
                    handled.add(k)
                    css.append(int(self.ast[ci]["rel"]))
            if css:
                checks.append(self.shortcut(ns, obj, css, d))
        for k, ci in enumerate(kids):
            if k in handled:
                continue
            ty = int(self.ast[ci]["type"])
            if ty == refsem.TTU:
                checks.append(self.check_ttu(ns, obj, ci, d))
            elif ty == refsem.CSS:
                checks.append((yield from self.check_css(ctx, ns, obj, int(self.ast[ci]["rel"]), d, nest + 1)))
            elif ty == refsem.REWRITE:
                checks.append((yield from self.check_rewrite(ctx, ns, obj, ci, d - 1, nest + 1)))
            elif ty == refsem.INVERT:
                checks.append((yield from self.check_inverted(ctx, ns, obj, ci, d, nest + 1)))
            else:
                return NOT_IMPL_F

        def f(ctx2, send):
            send((yield from (self._or if op == 0 else self._and)(ctx2, checks)))
        return f

    def shortcut(self, ns, obj, css, d):
        """the OR's computed-subject-set shortcut (rewrites.go:62-92) +
        TraverseSubjectSetRewrite (traverser.go:123-191)"""
        def f(ctx, send):
            yield None
            if ctx.cancelled:
                send((UNK, ERR_CANCELED))
                return
            rels = []
            for rel in css:
                ri, _ = self._relation_for(ns, rel)
                if self.strict and ri >= 0 and int(self.rels[ri]["rewrite"]) >= 0:
                    continue
                rels.append(rel)
            g = Group(self, ctx)
            if any(self._exists(ns, obj, rel) for rel in rels):
                yield from g.add(IS_F)  # SetIsMember
                send((yield from g.wait_result()))
                return
            for rel in css:
                cf = yield from self.check_is_allowed(ctx, ns, obj, rel, d - 1, True)
                yield from g.add(cf)
            send((yield from g.wait_result()))
        return f

    def check_css(self, ctx, ns, obj, rel, d, nest=0):  # checkComputedSubjectSet (rewrites.go:208-230)
        if d < 0:
            return UNK_F
        return (yield from self.check_is_allowed(ctx, ns, obj, rel, d, False, nest + 1))

    def check_inverted(self, ctx, ns, obj, ai, d, nest=0):  # checkInverted (rewrites.go:136-200)
        if d < 0:
            return UNK_F
        a = self.ast[ai]
        if int(a["child_count"]) != 1:
            return NOT_IMPL_F
        ci = int(self.children[int(a["child_begin"])])
        ty = int(self.ast[ci]["type"])
        if ty == refsem.TTU:
            check = self.check_ttu(ns, obj, ci, d)
        elif ty == refsem.CSS:
            check = yield from self.check_css(ctx, ns, obj, int(self.ast[ci]["rel"]), d, nest + 1)
        elif ty == refsem.REWRITE:
            check = yield from self.check_rewrite(ctx, ns, obj, ci, d, nest + 1)
        elif ty == refsem.INVERT:
            check = yield from self.check_inverted(ctx, ns, obj, ci, d, nest + 1)
        else:
            return NOT_IMPL_F

        def f(ctx2, send):
            inner = Future()
            self.sched.go(check(ctx2, inner.set))
            yield lambda: inner.done or ctx2.cancelled
            if not inner.done:
                send((UNK, ERR_CANCELED))
                return
            m, err = inner.value
            send(({IS: NOT, NOT: IS}.get(m, m), err))
        return f

    def check_ttu(self, ns, obj, ai, d):
        """checkTupleToSubjectSet (rewrites.go:242-293) + GetRelationTuples
        (relationtuples.go:207-247), one page"""
        if d < 0:
            return UNK_F
        a = self.ast[ai]
        rel, computed = int(a["rel"]), int(a["computed"])

        def f(ctx, send):
            g = Group(self, ctx)
            yield None
            if ctx.cancelled:  # the error path Adds the error and returns without a send (:270-273)
                yield from g.add(_const((UNK, ERR_CANCELED)))
                return
            for (kind, sid, sns, srel) in self.rows.get((ns, obj, rel), ()):
                if kind != 1:
                    continue
                cf = yield from self.check_is_allowed(ctx, sns, sid, computed, d - 1, False)
                yield from g.add(cf)
            send((yield from g.wait_result()))
        return f

    # -- binop.go --------------------------------------------------------------------------
    def _run(self, ctx, check):
        box = Future()
        yield from check(ctx, box.set)
        yield lambda: box.done or ctx.cancelled
        return box.value if box.done else (UNK, ERR_CANCELED)

    def _or(self, ctx, checks):  # binop.go:18-40
        for c in checks:
            r = yield from self._run(ctx, c)
            if decisive(r):
                return r
        return (NOT, 0)

    def _and(self, ctx, checks):  # binop.go:42-73
        if not checks:
            return (NOT, 0)
        for c in checks:
            r = yield from self._run(ctx, c)
            if r[1] != 0 or r[0] != IS:
                return (NOT, r[1])
        return (IS, 0)

    # -- engine.go:76-95 -------------------------------------------------------------------
    def check(self, q, seed: int, policy: str = "random"):
        """CheckRelationTuple for one query (refsem.QUERY_DT record) under one seeded schedule:
        (membership, error code, scheduler steps)"""
        self.sched = Sched(np.random.Generator(np.random.PCG64(seed)), policy)
        kind = int(q["kind"])
        self.subj = (kind, int(q["sid"]), int(q["sns"]), int(q["srel"])) if kind == 1 else (0, int(q["sid"]), 0, 0)
        d = int(q["depth"])
        if d <= 0 or self.max_depth < d:
            d = self.max_depth
        root = Ctx()
        out = Future()
        ns, obj, rel = int(q["ns"]), int(q["obj"]), int(q["rel"])

        def main():
            cf = yield from self.check_is_allowed(root, ns, obj, rel, d, False)
            self.sched.go(cf(root, out.set))
        self.sched.go(main())
        self.sched.run_until(lambda: out.done)
        return out.value[0], out.value[1], self.sched.steps

    def allowed(self, q, seed, policy="random"):
        """(allowed, error code), or None when the reference would not return (ReferenceCrash)"""
        try:
            m, err, _ = self.check(q, seed, policy)
        except ReferenceCrash:
            return None
        return int(err == 0 and m == IS), err
