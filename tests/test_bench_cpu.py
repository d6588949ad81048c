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


class _Ev:
    """Stand-in for a HIP event: elapsed_time in ms from a timestamp."""

    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def _worker_summary(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, REPO)
    import bench
    steps = 2
    # per step: layers exposed (1 + rank) ms, tail exposed 3 ms; 4 layer buckets + 2 tail buckets per step
    ev = [(_Ev(0.0), _Ev(1.0 + rank), _Ev(4.0 + rank)) for _ in range(steps)]
    log = [(64 << 20, False)] * 4 * steps + [(100 << 20, True), (50 << 20, True)] * steps
    out[rank] = bench.exchange_summary(ev, log, steps, t_rank=0.5 + 0.1 * rank, pg=dist.group.WORLD, world=world,
                                       device="cpu")
    dist.destroy_process_group()


def test_distributed_fields():
    """the JSON line's `distributed` object carries the bytes exchanged per step (and the tail's
    share), the per-rank step times and their spread, and the exposed exchange split into the per-layer buckets and
    the tail bucket -- computed here on 2 gloo ranks from stand-in events."""
    import torch.multiprocessing as mp
    world = 2
    out = mp.Manager().dict()
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_worker_summary, args=(world, port, out), nprocs=world, join=True)
    d0, d1 = out[0], out[1]
    # the gathered per-rank lists agree on every rank; the exposed times are each rank's own (rank 0 prints)
    assert d0["rank_step_ms"] == d1["rank_step_ms"] and d0["rank_exchange_exposed_ms"] == d1["rank_exchange_exposed_ms"]
    assert d1["exchange_exposed_layers_ms_per_step"] == 2.0
    assert d0["backend"] == "gloo" and d0["world_size"] == 2
    assert d0["exchange_bytes_per_step"] == 4 * (64 << 20) + (150 << 20)
    assert d0["exchange_tail_bytes_per_step"] == 150 << 20
    assert d0["exchange_buckets_per_step"] == 6
    assert d0["ring_bytes_per_gpu_per_step"] == d0["exchange_bytes_per_step"]      # 2 (N-1)/N = 1 at N = 2
    assert d0["exchange_exposed_layers_ms_per_step"] == 1.0 and d0["exchange_exposed_tail_ms_per_step"] == 3.0
    assert d0["exchange_exposed_ms_per_step"] == 4.0
    assert d0["rank_step_ms"] == [250.0, 300.0] and d0["rank_step_ms_spread"] == 50.0
    assert d0["rank_exchange_exposed_ms"] == [4.0, 5.0]


def test_single_rank_summary():
    sys.path.insert(0, REPO)
    import bench
    d = bench.exchange_summary(None, None, 3, 1.0, None, 1, "cpu")
    assert d == dict(backend=None, world_size=1, exchange=None)
