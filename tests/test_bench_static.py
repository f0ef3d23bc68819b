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
