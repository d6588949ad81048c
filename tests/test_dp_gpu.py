"""Data-parallel step on the GPU: 2 ranks sharing cuda:0 over gloo (the 1-GPU box; on 8 GPUs the
same code runs over RCCL).  The per-layer gradient exchange starts inside the backward
(Backward.on_ready -> async all-reduce of each finished layer's slice) and the rest follows at the
end; after one optimizer step both ranks hold identical weights, equal (fp32 summation order aside:
1e-6 relative on the update) to one process accumulating the two half-batches (DDP mean semantics,
SURVEY.md §8e)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import sys
    for p in (REPO, os.path.join(REPO, "taiwan-whisper_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from conftest import load_golden
    from oracle.weights import CONFIGS, make_weights
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    tc = WhisperConfig(**cfg)
    mk = lambda seed, dt: WhisperForConditionalGeneration.from_state_dict(
        tc, {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed).items()}, dtype=dt)
    g = load_golden("micro_step")
    return mk, g


def _batch(g, lo, hi):
    return {"input_features": torch.from_numpy(g["feats"][lo:hi]).cuda(),
            "decoder_input_ids": torch.from_numpy(g["dec"][lo:hi]).cuda(),
            "labels": torch.from_numpy(g["lab"][lo:hi]).cuda()}


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    mk, g = _setup()
    from tw.distill import DistillationTrainer
    s, t = mk(1, torch.float32), mk(2, torch.bfloat16)
    tr = DistillationTrainer(s, t, learning_rate=1e-3, freeze_encoder=False, dp_bucket_mb=1,
                             process_group=torch.distributed.group.WORLD)
    launched = []
    orig = tr._grad_ready
    tr._grad_ready = lambda p: (launched.append(p), orig(p))
    B = g["feats"].shape[0]
    h = B // world
    tr.train_step(_batch(g, rank * h, (rank + 1) * h))
    torch.cuda.synchronize()
    out[rank] = (s.store.p32.cpu().clone(), list(launched))
    torch.distributed.destroy_process_group()


def test_dp_two_ranks_equal_accumulation():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    p0, l0 = out[0]
    p1, l1 = out[1]
    assert torch.equal(p0, p1)
    # every decoder and encoder layer started its exchange inside the backward
    assert any(p.startswith("model.decoder.layers.") for p in l0) and any(p.startswith("model.encoder.layers.")
                                                                          for p in l0)
    # single process, the two halves accumulated (loss / 2 each) = DDP mean of per-rank gradients
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    mk, g = _setup()
    from tw.distill import DistillationTrainer
    s, t = mk(1, torch.float32), mk(2, torch.bfloat16)
    init = s.store.p32.clone()
    tr = DistillationTrainer(s, t, learning_rate=1e-3, freeze_encoder=False, gradient_accumulation_steps=2)
    B = g["feats"].shape[0]
    h = B // world
    tr.train_step(_batch(g, 0, h))
    tr.train_step(_batch(g, h, 2 * h))
    torch.cuda.synchronize()
    ref = s.store.p32.cpu()
    d_dp, d_acc = p0 - init.cpu(), ref - init.cpu()
    rel = float((d_dp - d_acc).norm() / d_acc.norm())
    assert rel < 1e-3, rel


def _worker_overlap(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    mk, g = _setup()
    from tw.distill import DistillationTrainer
    B = g["feats"].shape[0]
    h = B // world
    res = {}
    for overlap in (False, True):
        s, t = mk(1, torch.float32), mk(2, torch.bfloat16)
        tr = DistillationTrainer(s, t, learning_rate=1e-3, freeze_encoder=True, dp_bucket_mb=1,
                                 process_group=torch.distributed.group.WORLD, overlap_update=overlap)
        for it in range(3):
            lo = (rank * h + it) % B
            tr.train_step(_batch(g, lo, lo + min(h, B - lo)))
            if overlap:
                assert tr._update is not None        # the update waits for the next step's encoder
        sd = tr.state_dict()                          # flushes
        assert tr._update is None and tr.step == 3
        torch.cuda.synchronize()
        res[overlap] = (s.store.p32.cpu().clone(), sd["exp_avg"].cpu().clone(), sd["exp_avg_sq"].cpu().clone())
    out[rank] = res
    torch.distributed.destroy_process_group()


def test_dp_deferred_update_bit_identical():
    """The deferred update (exchange tail beside the next step's frozen-encoder forward, then clip +
    AdamW) gives bit-identical weights and moments to the in-step update after 3 steps, on both ranks."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker_overlap, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        a, b = out[r][False], out[r][True]
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    assert torch.equal(out[0][True][0], out[1][True][0])


def _worker_rccl(rank, world, port, out):
    """One rank on a real `nccl` (= RCCL) process group with the exchange forced on (force_exchange): per-layer async
    all-reduces issued from the backward hook, the tail, Work.wait() on the compute stream and the deferred AdamW
    (overlap_update) all run on the backend of the 8-GPU node; the same steps without a process group beside it."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    mk, g = _setup()
    from tw.distill import DistillationTrainer
    B = g["feats"].shape[0]
    res = {}
    for dp in (True, False):
        s, t = mk(1, torch.float32), mk(2, torch.bfloat16)
        kw = dict(process_group=torch.distributed.group.WORLD, force_exchange=True, overlap_update=True) if dp else {}
        tr = DistillationTrainer(s, t, learning_rate=1e-3, freeze_encoder=True, dp_bucket_mb=1, **kw)
        launched = []
        if dp:
            tr.exchange_log, tr.exchange_events = [], []
            orig = tr._grad_ready
            tr._grad_ready = lambda p, orig=orig: (launched.append(p), orig(p))
        for it in range(3):
            tr.train_step(_batch(g, it % B, it % B + 1))
            if dp:
                assert tr._update is not None        # the update waits for the next step's encoder
        sd = tr.state_dict()                          # flushes
        torch.cuda.synchronize()
        res[dp] = (s.store.p32.cpu().clone(), sd["exp_avg"].cpu().clone(), sd["exp_avg_sq"].cpu().clone(),
                   list(launched), list(tr.exchange_log or []), len(tr.exchange_events or []),
                   torch.distributed.get_backend() if dp else None)
    out[rank] = res
    torch.distributed.destroy_process_group()


def test_dp_rccl_one_rank_bit_identical():
    """the RCCL code path on one GPU.  DistillationTrainer on an `nccl` process group of world size
    1 with the exchange forced on and the deferred update: after 3 steps the weights and AdamW moments are
    bit-identical to the trainer without a process group (an all-reduce over one rank is the identity), every decoder
    layer's exchange started inside the backward, and the tail went out after it."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = mp.Manager().dict()
    mp.spawn(_worker_rccl, args=(1, _free_port(), out), nprocs=1, join=True)
    dp, ref = out[0][True], out[0][False]
    for x, y in zip(dp[:3], ref[:3]):
        assert torch.equal(x, y)
    launched, log, nwait, backend = dp[3], dp[4], dp[5], dp[6]
    assert backend == "nccl"
    assert any(p.startswith("model.decoder.layers.") for p in launched)
    assert any(not tail for _, tail in log) and any(tail for _, tail in log)
    assert nwait == 3
