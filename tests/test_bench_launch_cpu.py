"""bench.py's N-GPU entry point on the CPU: ``python bench.py --gpus 2`` outside a
torch.distributed.run environment starts 2 ranks itself (a child torch.distributed.run on
127.0.0.1), every rank joins one process group, and the parent exits with the child's code.
``--launch-check`` stops each rank after the rendezvous, before any GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lines(out):
    res = []
    for line in out.splitlines():
        i = line.find('{"launch_check"')
        while i >= 0:                       # ranks may print on one line without a newline between
            j = line.index("}", i) + 1
            res.append(json.loads(line[i:j]))
            i = line.find('{"launch_check"', j)
    return res


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_n_spawns_n_ranks(n):
    """--gpus 2 and --gpus 8 (the driver's node size): n ranks over gloo on the CPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    got = _lines(p.stdout)
    assert sorted(r["rank"] for r in got) == list(range(n)), p.stdout
    assert all(r["world_size"] == n and r["gpus"] == n for r in got)


def test_driver_style_torchrun_8_ranks():
    """The driver's own launch (python -m torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8),
    CPU-only: each process is one rank of the 8 (no nested launcher)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "bench.py"),
                        "--gpus", "8", "--launch-check"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    got = _lines(p.stdout)
    assert sorted(r["rank"] for r in got) == list(range(8)), p.stdout


def test_gpus_1_is_one_process():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-check"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0
    assert _lines(p.stdout) == [{"launch_check": True, "rank": 0, "world_size": 1, "gpus": 1}]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


def test_baseline_procs_policy():
    sys.path.insert(0, ROOT)
    import bench
    phys, aff = bench.host_cores()
    assert phys >= 1 and aff >= 1
    procs, p2, a2 = bench.baseline_procs()
    assert (p2, a2) == (phys, aff) and 1 <= procs <= min(phys, aff, 16)
    assert bench.baseline_procs(3)[0] == 3
    ex = bench._extrapolate(1000.0, 4, 8, 0.0, 4096, 5)
    assert abs(ex["env_only"] - 2000.0) < 1e-9 and ex["cores"] == 8
    # the measured 1 -> n per-process decline is applied again from n to the physical cores
    ex = bench._extrapolate(1000.0, 4, 8, 0.0, 4096, 5, eff=186.7 / 212.7)
    assert abs(ex["env_only"] - 2000.0 * 186.7 / 212.7) < 1e-9
