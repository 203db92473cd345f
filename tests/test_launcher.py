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
