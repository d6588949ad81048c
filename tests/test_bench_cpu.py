"""bench.py's multi-GPU entry: `python bench.py --gpus N` with no launcher starts the N ranks
itself (torch.distributed.run, before any GPU call), and a launcher whose WORLD_SIZE differs from --gpus is refused
with a non-zero exit -- checked here without a GPU (the refusal happens before the device is touched)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update({k: str(v) for k, v in kw.items()})
    return env


def test_gpus_without_launcher_starts_the_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3"], env=_env(TW_BENCH_PRINT_LAUNCH=1),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index(BENCH) + 1:] == ["--gpus", "2", "--steps", "3"]


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE=2, RANK=0, LOCAL_RANK=0),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_world_size_mismatch_under_the_launcher():
    """The driver's own command shape (torch.distributed.run, 2 ranks, 127.0.0.1) with a wrong --gpus: every rank
    refuses before touching a device, so the launcher fails."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", "29613", BENCH, "--gpus", "3"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
