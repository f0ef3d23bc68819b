"""CPU: a pipeline that fails inside bench.py's timed region stops the run
(a worker thread died with hipMalloc OOM, the others kept
going and the rate still divided all --steps by the elapsed time).  The
stubs stand in for torch's stream plumbing and the library's cover/search."""
import contextlib
import os
import subprocess
import sys
import textwrap
import threading
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _Stream:
    def synchronize(self):
        pass

    def wait_event(self, ev):
        pass


class _Event:
    def record(self, stream=None):
        pass


def fake_torch():
    cuda = types.SimpleNamespace(stream=lambda s: contextlib.nullcontext(), current_stream=lambda: _Stream(),
                                 Stream=_Stream, Event=_Event)
    return types.SimpleNamespace(cuda=cuda)


class FailingLib:
    """cover() always works; search() raises on the `fail_at`-th call made
    from a thread other than the main one (a worker pipeline's context)."""

    def __init__(self, fail_at=2):
        self.fail_at = fail_at
        self.calls = 0
        self.done = 0
        self.lock = threading.Lock()

    def cover(self, ctx, d_q):
        return ("cells", ctx)

    def search(self, ctx, index, cells, *qargs):
        with self.lock:
            self.calls += 1
            bad = ctx == "worker" and self.calls >= self.fail_at
        if bad:
            raise RuntimeError("dssg error 3: hipMalloc of 2562523140 bytes: out of memory")
        with self.lock:
            self.done += 1


def test_replica_steps_raise_when_a_worker_fails():
    D = FailingLib(fail_at=2)
    workers = [("worker", _Stream()), ("worker", _Stream())]
    with pytest.raises(bench.StepFailure, match="out of memory"):
        bench.replica_steps(fake_torch(), D, "main", workers, None, None, (), steps=20)
    assert D.done < 20


def test_replica_steps_all_finish_without_faults():
    D = FailingLib(fail_at=10**9)
    bench.replica_steps(fake_torch(), D, "main", [("worker", _Stream())], None, None, (), steps=17)
    assert D.done == 17


def test_cover_ahead_steps_raise_when_a_cover_pipeline_fails():
    class CoverFails(FailingLib):
        def cover(self, ctx, d_q):
            if ctx == "worker":
                raise RuntimeError("dssg error 3: cover out of memory")
            return ("cells", ctx)
    D = CoverFails()
    seen = []
    with pytest.raises(bench.StepFailure, match="cover out of memory"):
        bench.cover_ahead_steps(fake_torch(), D, "main", [("worker", _Stream())], None, 5, seen.append)
    assert seen == []


def test_cover_ahead_steps_search_failure_releases_cover_threads():
    D = FailingLib()
    calls = []

    def search_fn(c):
        calls.append(c)
        if len(calls) == 2:
            raise RuntimeError("exchange failed")
    with pytest.raises(RuntimeError, match="exchange failed"):
        bench.cover_ahead_steps(fake_torch(), D, "main", [("worker", _Stream()), ("worker", _Stream())], None, 8,
                                search_fn)
    assert len(calls) == 2


def test_bench_process_exits_nonzero_on_a_failed_pipeline():
    """The same failure in a bench.py process: non-zero exit, no result line
    on stdout."""
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
        import bench, test_bench_failure as T
        bench.keep_stdout_for_json()
        bench.replica_steps(T.fake_torch(), T.FailingLib(2), "main", [("worker", T._Stream())], None, None, (), 10)
        bench.emit({{"metric": "should not be printed"}})
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "StepFailure" in r.stderr
    assert r.stdout.strip() == ""
