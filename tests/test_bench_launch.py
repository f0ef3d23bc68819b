"""CPU: `bench.py --gpus N` with no launcher starts N rank processes itself
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one rendezvous port) before
anything touches a GPU, and relays rank 0's result line (VERDICT r2 item 1:
the driver runs `python3 bench.py --gpus N` for N = 1 as well)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_probe(tmp_path, n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-probe",
                        str(tmp_path)], env=env, capture_output=True, text=True, timeout=120)
    return r


def test_gpus_2_spawns_two_ranks(tmp_path):
    r = run_probe(tmp_path, 2)
    assert r.returncode == 0, r.stderr
    recs = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    assert [x["rank"] for x in recs] == ["0", "1"]
    assert [x["local_rank"] for x in recs] == ["0", "1"]
    assert all(x["world_size"] == "2" for x in recs)
    assert all(x["master_addr"] == "127.0.0.1" for x in recs)
    assert recs[0]["master_port"] == recs[1]["master_port"]
    assert recs[0]["pid"] != recs[1]["pid"]
    assert not any(x["torch_imported"] for x in recs)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["launch_probe"]["rank"] == "0"


def test_gpus_8_spawns_eight_ranks(tmp_path):
    r = run_probe(tmp_path, 8)
    assert r.returncode == 0, r.stderr
    ranks = sorted(int(json.load(open(tmp_path / f"rank{k}.json"))["rank"]) for k in range(8))
    assert ranks == list(range(8))


def test_gpus_1_runs_in_process(tmp_path):
    r = run_probe(tmp_path, 1)
    assert r.returncode == 0, r.stderr
    rec = json.load(open(tmp_path / "rank0.json"))
    assert rec["world_size"] is None and rec["pid"] != os.getpid()


def test_under_a_launcher_no_second_spawn(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-probe",
                        str(tmp_path)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(tmp_path)) == ["rank1.json"]
