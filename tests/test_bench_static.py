"""CPU: bench.py's functions reference no undefined names.  The multi-GPU
report path (sharded_report) only runs under torchrun on a GPU node, so a
name error there would otherwise surface first in the driver's scaling run."""
import ast
import builtins
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def undefined_names(path):
    tree = ast.parse(open(path).read())
    module = {n.name for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef))}
    module |= {a.asname or a.name.split(".")[0] for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom))
               for a in n.names}
    module |= {t.id for n in tree.body if isinstance(n, ast.Assign) for t in n.targets if isinstance(t, ast.Name)}
    bad = []
    for fn in [n for n in tree.body if isinstance(n, ast.FunctionDef)]:
        known = {a.arg for a in fn.args.args + fn.args.kwonlyargs}
        if fn.args.vararg:
            known.add(fn.args.vararg.arg)
        if fn.args.kwarg:
            known.add(fn.args.kwarg.arg)
        for n in ast.walk(fn):
            if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
                known.add(n.id)
            elif isinstance(n, (ast.Import, ast.ImportFrom)):
                known |= {a.asname or a.name.split(".")[0] for a in n.names}
            elif isinstance(n, (ast.FunctionDef, ast.Lambda)) and n is not fn:
                known |= {a.arg for a in n.args.args}
                if isinstance(n, ast.FunctionDef):
                    known.add(n.name)
            elif isinstance(n, ast.ExceptHandler) and n.name:
                known.add(n.name)
        for n in ast.walk(fn):
            if (isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id not in known and n.id not in module
                    and not hasattr(builtins, n.id)):
                bad.append((fn.name, n.id, n.lineno))
    return bad


def test_bench_has_no_undefined_names():
    assert undefined_names(os.path.join(ROOT, "bench.py")) == []


def _result_dict(fn_name):
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == fn_name)
    for n in ast.walk(fn):
        if isinstance(n, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "result" for t in n.targets) \
                and isinstance(n.value, ast.Dict):
            return {k.value: v for k, v in zip(n.value.keys, n.value.values) if isinstance(k, ast.Constant)}
    raise AssertionError(f"no result dict in {fn_name}")


def test_every_line_carries_baseline_parity_and_traffic():
    """Both result lines (replica: main, sharded N > 1: sharded_report) carry
    a computed cpu_baseline, parity and roofline.traffic -- never a literal
    None (the N > 1 lines had cpu_baseline None)."""
    for fn in ("main", "sharded_report"):
        res = _result_dict(fn)
        for key in ("cpu_baseline", "parity", "roofline", "value", "metric", "config"):
            assert key in res, (fn, key)
        for key in ("cpu_baseline", "parity"):
            assert not (isinstance(res[key], ast.Constant) and res[key].value is None), (fn, key)
        roof = {k.value: v for k, v in zip(res["roofline"].keys, res["roofline"].values)}
        assert "traffic" in roof and not (isinstance(roof["traffic"], ast.Constant) and roof["traffic"].value is None)
    assert "exchanged" in _result_dict("sharded_report")


def test_sharded_leg_attached_to_the_replica_line():
    """N > 1 replica runs time the cell-range shards in the same ranks
    (VERDICT r5 item 2): main() hands the replica index to sharded_leg and
    puts its record under result["sharded"]; the record carries the rate,
    the phases and oracle parity on every rank."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'result["sharded"] = rec' in src
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "sharded_leg")
    text = ast.get_source_segment(src, fn)
    for key in ('"value"', '"ms_per_step"', '"oracle_all_ranks_equal"', '"all_ranks_equal"',
                '"phase_ms_max_over_ranks"', 'rec["error"]'):
        assert key in text, key


def test_sharded_leg_watchdog_keeps_the_replica_line(tmp_path):
    """A sharded-leg stage past its limit (a hung collective) ends the rank
    with status 0 and rank 0 prints the finished replica line, with
    sharded.error set -- the replica measurement is never lost."""
    import json
    import subprocess
    import sys
    code = ("import sys, time; sys.path.insert(0, %r); import bench; bench.LEG_LIMIT_S = 0.3; "
            "bench._PENDING[0] = {'metric': 'm', 'value': 1.0}; bench._PENDING[1] = 0; "
            "bench.heartbeat(every=0.1); bench.stage('sharded leg: timed steps'); time.sleep(30)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and "exceeded" in d["sharded"]["error"]
