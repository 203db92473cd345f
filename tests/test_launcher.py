"""CPU, world_size 2: bench.py's multi-GPU launcher path itself.

`python bench.py --gpus 2 --dry-run` starts two ranks through
torch.distributed.run from a parent that makes no GPU call; the ranks
exchange a 128-byte communicator id through the job's rendezvous directory
(what rank 0's ncclGetUniqueId takes on a GPU node) and compute their config[2]
shards with the library's own cess_bls_shard_range.  Rank 0 checks that the
shards tile the batch and that every rank saw the same id."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus, n=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run"]
    if n:
        cmd += ["--n", str(n)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


def test_launcher_two_ranks_config2():
    rec = _run(2)
    assert rec["n_gpus"] == 2 and rec["sigs_per_gpu"] == 1 << 21 and rec["n_total"] == 1 << 22
    assert rec["cover_ok"] and rec["same_comm_id"]
    assert sorted(s["rank"] for s in rec["shards"]) == [0, 1]
    for s in rec["shards"]:
        assert s["end"] - s["begin"] == 1 << 21 and s["wpr"] == (1 << 21) // 64


def test_launcher_three_ranks_ragged():
    rec = _run(3, n=1000)
    assert rec["n_gpus"] == 3 and rec["cover_ok"] and rec["same_comm_id"]


def _run_fail(gpus, env_extra, extra_env_rank=None):
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    errs = [json.loads(x) for x in r.stderr.splitlines() if x.startswith("{")]
    return r, errs


def test_launcher_fails_fast_with_fewer_devices_than_ranks():
    """A node with fewer visible GPUs than ranks: the launcher parent exits
    non-zero with one JSON error line BEFORE starting any rank (no communicator
    to hang on), counting devices without a HIP call (CESS_BENCH_DEVICE_COUNT
    stands in for the node's KFD topology here)."""
    r, errs = _run_fail(4, {"CESS_BENCH_DEVICE_COUNT": "2"})
    assert r.returncode == 4, (r.stdout[-2000:], r.stderr[-2000:])
    assert errs and errs[0]["error"] == "devices" and errs[0]["need"] == 4 and errs[0]["visible"] == 2
    assert errs[0]["where"] == "launcher"
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]   # no result line


def test_rank_fails_fast_under_external_torchrun():
    """Under the driver's own torchrun there is no launcher parent of ours:
    each rank counts the devices before any context or communicator exists
    and exits non-zero, so the job ends at once."""
    env = dict(os.environ, CESS_BENCH_DEVICE_COUNT="1", WORLD_SIZE="2", RANK="1", LOCAL_RANK="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 4, (r.stdout[-2000:], r.stderr[-2000:])
    errs = [json.loads(x) for x in r.stderr.splitlines() if x.startswith("{")]
    assert errs and errs[0]["error"] == "devices" and errs[0]["where"] == "rank" and errs[0]["rank"] == 1


def test_node_gpu_count_reads_visible_devices(monkeypatch):
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setenv("CESS_BENCH_DEVICE_COUNT", "3")
    assert bench.node_gpu_count() == 3
    monkeypatch.delenv("CESS_BENCH_DEVICE_COUNT")
    n = bench.node_gpu_count()
    assert n is None or n >= 0   # no KFD topology in a CPU container: None
    if n is not None:
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
        assert bench.node_gpu_count() <= 1
