"""Closure-table worker pool on the CPU (robustgrape_amd/tables.py): the pool's tables equal the
serial ones, and equal them again after the closures' captured state changed between calls
(workers receive the problem by value with every call); the chunk byte cap."""
import numpy as np

from tests import problems as P


def test_pool_tables_follow_the_closures_current_state():
    from robustgrape_amd import tables as TB
    fp = P.sym_problem(6, errors=("amp",), device=False)
    up = fp.unitary_problem
    base = up.H0
    state = {"scale": 1.0}

    def h0(t, p, xa):  # reads a captured mutable: the reference calls it live at every site
        return state["scale"] * np.asarray(base(t, p, xa))

    fp2 = fp.replace(unitary_problem=up.replace(H0=h0))
    X = np.stack([P.random_x(6, s) for s in range(3)])
    W = TB.TableWorkers(2)
    sh, su = TB.table_shapes(fp2, len(X), 1)
    tabs = TB.SharedTables(sh, su)
    try:
        for scale in (1.0, 1.7, 1.0):
            state["scale"] = scale
            shipped = W.prepare(fp2)
            assert shipped is not None
            for r in W.submit(shipped, 1, tabs, X, range(len(X))):
                r.get(timeout=120)
            H, U0 = TB.host_tables(fp2, X, 1)
            np.testing.assert_array_equal(tabs.H, H)
            np.testing.assert_array_equal(tabs.U0, U0)
        # one evaluation split by time steps over the workers
        tabs1 = TB.SharedTables(*TB.table_shapes(fp2, 1, 1))
        try:
            state["scale"] = 0.5
            for r in W.submit(W.prepare(fp2), 1, tabs1, X, range(1)):
                r.get(timeout=120)
            H, U0 = TB.host_tables(fp2, X[:1], 1)
            np.testing.assert_array_equal(tabs1.H, H)
            np.testing.assert_array_equal(tabs1.U0, U0)
        finally:
            W.release(tabs1)
            tabs1.close()
    finally:
        W.release(tabs)
        tabs.close()
        W.close()


def test_worker_errors_reach_the_caller():
    """A closure that raises inside a worker: the error surfaces in get()."""
    from robustgrape_amd import tables as TB
    fp = P.sym_problem(4, device=False)
    up = fp.unitary_problem

    def h0(t, p, xa):
        if t == 3:
            raise ValueError("closure failed at step 3")
        return up.H0(t, p, xa)

    bad = fp.replace(unitary_problem=up.replace(H0=h0))
    X = P.random_x(4, 2)[None, :]
    W = TB.TableWorkers(2)
    tabs = TB.SharedTables(*TB.table_shapes(bad, 1, 1))
    try:
        rs = W.submit(W.prepare(bad), 1, tabs, X, range(1))
        errs = 0
        for r in rs:
            try:
                r.get(timeout=120)
            except ValueError as e:
                assert "step 3" in str(e)
                errs += 1
        assert errs >= 1
    finally:
        tabs.close()
        W.close()


def test_table_chunk_cap_by_bytes(monkeypatch):
    from robustgrape_amd import tables as TB
    fp = P.sym_problem(8, errors=("amp", "freq"), device=False)
    sh, su = TB.table_shapes(fp, 1, 1)
    per = (int(np.prod(sh)) + int(np.prod(su))) * 16
    assert TB.table_batch_cap(fp, 1) == max(1, TB.TABLE_CHUNK_BYTES // per)
    monkeypatch.setenv("GRAPE_TABLE_CHUNK_MB", str(3 * per / 2 ** 20))
    assert TB.table_batch_cap(fp, 1) == 3
    monkeypatch.setenv("GRAPE_TABLE_CHUNK_MB", "0")
    assert TB.table_batch_cap(fp, 1) == 1


UNGUARDED_SCRIPT = """
import os, sys
import numpy as np
sys.path.insert(0, {root!r})
with open({marker!r}, "a") as fh:      # top-level code: must run once, in this process only
    fh.write("%d\\n" % os.getpid())
from robustgrape_amd import tables as TB
from tests import problems as P
fp = P.sym_problem(4, device=False)
up = fp.unitary_problem
base = up.H0
h0 = lambda t, p, xa: 1.0 * np.asarray(base(t, p, xa))   # a __main__ closure (shipped by value)
fp2 = fp.replace(unitary_problem=up.replace(H0=h0))
X = np.stack([P.random_x(4, s) for s in range(2)])
W = TB.TableWorkers(2)
tabs = TB.SharedTables(*TB.table_shapes(fp2, len(X), 1))
for r in W.submit(W.prepare(fp2), 1, tabs, X, range(len(X))):
    r.get(timeout=120)
H, U0 = TB.host_tables(fp2, X, 1)
assert np.array_equal(tabs.H, H) and np.array_equal(tabs.U0, U0)
# a worker dies: the pool's replacement starts through the same hidden-main context (ADVICE r4).
# (The worker exits inside a task: a worker killed while idle may hold the task queue's read lock,
# which would stall the pool forever -- multiprocessing's own limitation, not the table workers'.)
import os as _os, time as _time
before = {{p.pid for p in W.pool._pool}}
W.pool.apply_async(_os._exit, (0,))
for _ in range(600):
    now = {{p.pid for p in W.pool._pool if p.is_alive()}}
    if len(now) == len(before) and now != before:
        break
    _time.sleep(0.05)
assert {{p.pid for p in W.pool._pool}} != before
for r in W.submit(W.prepare(fp2), 1, tabs, X, range(len(X))):
    r.get(timeout=120)
assert np.array_equal(tabs.H, H)
W.release(tabs)
tabs.close()
W.close()
print("UNGUARDED-OK")
"""


def test_pool_from_a_script_without_main_guard(tmp_path):
    """spawned workers must not re-run an unguarded user script's top-level code
    (robustgrape_amd/tables.py _main_hidden)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    marker = tmp_path / "marker.txt"
    script = tmp_path / "user_script.py"
    script.write_text(UNGUARDED_SCRIPT.format(root=root, marker=str(marker)))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "UNGUARDED-OK" in r.stdout
    assert len(marker.read_text().split()) == 1, marker.read_text()
