"""Data-parallel semantics on CPU with gloo, world_size 2 (no GPU needed).

1. The product's gradient exchange (`DistillationTrainer.all_reduce_grads`, bucketed async SUM of
   the flat fp32 gradient; per-layer ranges launched early during the backward, the remainder at the
   end) equals the DDP mean of per-rank gradients, for bucket sizes and early ranges that split the
   buffer unevenly: world 2 (1/world folded into the loss gradient, exact) and world 3 (each slice
   scaled by fp32(1/3) before its SUM, torch Reducer's order -- bit-exact against that recipe).
2. SURVEY.md §8(e) semantics on the oracle step: 2 ranks x half batch with DDP mean == 1 process
   accumulating the two halves with loss / 2 each (per-rank token normalisation kept).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_allreduce(rank, world, port, out):
    fold = world & (world - 1) == 0
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "taiwan-whisper_amd"))
    from tw.distill import DistillationTrainer
    _init(rank, world, port)
    n = 10_007
    g = torch.Generator().manual_seed(rank)
    local = torch.randn(n, generator=g)

    import types

    class Stub:
        pass
    st = Stub()
    st.s = Stub()
    st.bw = Stub()
    # power-of-two world: the trainer folds 1/world into the loss gradient; otherwise the exchange scales
    st.s.grad = local / world if fold else local.clone()
    st.world, st.pg, st.bucket, st.fold_world, st.dp = world, dist.group.WORLD, 3001, fold, world > 1
    st.scaler = None
    for name in ("_launch", "launch_grad_exchange", "wait_grad_exchange"):
        setattr(st, name, types.MethodType(getattr(DistillationTrainer, name), st))
    # two "layers" finished during the backward start their exchange early (out of order, uneven
    # sizes); all_reduce_grads then covers the gaps and waits for everything
    st._pending, st._reduced = [], []
    st._launch(6000, 9000)
    st._launch(100, 2500)
    DistillationTrainer.all_reduce_grads(st)
    assert st._pending == [] and st._reduced == []
    out[rank] = st.s.grad.clone()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_is_ddp_mean(world):
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker_allreduce, args=(world, port, out), nprocs=world, join=True)
    n = 10_007
    g = [torch.randn(n, generator=torch.Generator().manual_seed(r)) for r in range(world)]
    # torch DDP (Reducer::mark_variable_ready_dense without a comm hook): bucket = grad * (1/world), SUM
    scaled = [x * (1.0 / world) for x in g]
    for r in range(world):
        got = out[r]
        # every rank holds the same bits; vs the DDP recipe: a 3-term fp32 sum in some order (1 ulp)
        assert torch.equal(got, out[0])
        assert torch.allclose(got, scaled[0] + scaled[1] + (scaled[2] if world == 3 else 0), rtol=2e-7, atol=1e-7)
        if world == 3:
            # not the folded variant's bits in general (a rank-local 1/3 before vs after rounding)
            assert torch.allclose(got, sum(g) / 3, rtol=1e-6, atol=1e-6)


def _worker_oracle(rank, world, port, out):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    from oracle import distill_ref, labels as L
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    _init(rank, world, port)
    torch.set_num_threads(2)
    cfg = CONFIGS["micro"]
    ps = to_torch(make_weights(cfg, 1))
    names = [n for n in ps if n.startswith("model.decoder.layers.1")]
    for n in names:
        ps[n].requires_grad_(True)
    S, T = Ref(cfg, ps), Ref(cfg, to_torch(make_weights(cfg, 2)))
    feats = torch.from_numpy(np.random.default_rng(0).standard_normal((4, 80, 3000)).astype(np.float32) * 0.3)
    dec, lab = L.collate(L.synthetic_label_lists(4, seed=3))
    dec, lab = torch.from_numpy(dec), torch.from_numpy(lab)
    sl = slice(2 * rank, 2 * rank + 2)       # batch -> rank mapping: micro-batch k*N + r
    distill_ref.train_step(S, T, feats[sl], dec[sl], lab[sl])
    flat = torch.cat([ps[n].grad.flatten() for n in names])
    dist.all_reduce(flat)
    out[rank] = flat / world
    dist.destroy_process_group()


def test_dp_mean_equals_accumulation_on_oracle():
    world = 2
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker_oracle, args=(world, port, out), nprocs=world, join=True)
    # single process, two micro-batches, loss / 2 each (Accelerate gradient accumulation)
    from oracle import distill_ref, labels as L
    from oracle.weights import CONFIGS, make_weights
    from oracle.whisper_ref import Ref, to_torch
    cfg = CONFIGS["micro"]
    ps = to_torch(make_weights(cfg, 1))
    names = [n for n in ps if n.startswith("model.decoder.layers.1")]
    for n in names:
        ps[n].requires_grad_(True)
    S, T = Ref(cfg, ps), Ref(cfg, to_torch(make_weights(cfg, 2)))
    feats = torch.from_numpy(np.random.default_rng(0).standard_normal((4, 80, 3000)).astype(np.float32) * 0.3)
    dec, lab = L.collate(L.synthetic_label_lists(4, seed=3))
    dec, lab = torch.from_numpy(dec), torch.from_numpy(lab)
    acc = None
    for k in range(2):
        for n in names:
            ps[n].grad = None
        sl = slice(2 * k, 2 * k + 2)
        distill_ref.train_step(S, T, feats[sl], dec[sl], lab[sl])
        g = torch.cat([ps[n].grad.flatten() for n in names]) / 2
        acc = g if acc is None else acc + g
    for r in range(world):
        assert torch.allclose(out[r], acc, rtol=1e-5, atol=1e-7)


def _worker_eval_gather(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "taiwan-whisper_amd"))
    from tw.dataset import shard_micro_batches
    from tw.run_distillation import gather_eval_rows
    _init(rank, world, port)
    n_items, B = 11, 2
    mbs, real = shard_micro_batches(n_items, B, rank, world, with_real=True)
    # a "prediction" row per item that names the item, so duplicates would be visible
    rows = [(bi, [[i, 7] for i in mb[:k]], [[i] for i in mb[:k]]) for bi, (mb, k) in enumerate(zip(mbs, real))]
    out[rank] = gather_eval_rows(rows, world)
    dist.destroy_process_group()


def test_eval_gather_drops_even_batches_duplicates():
    """Eval predictions are gathered like accelerate's gather_for_metrics: every item once, in
    batch-major / rank order (11 items, B = 2, world 3: the last group wraps 1 item around)."""
    world = 3
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker_eval_gather, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        preds, labels = out[r]
        assert [p[0] for p in preds] == list(range(11))
        assert labels == [[i] for i in range(11)]


def _worker_deferred(rank, world, port, out):
    """optimizer_step with overlap_update launches the exchange and applies nothing; flush() waits for it
    and applies clip + AdamW once with the step's own lr / t; a second flush is a no-op."""
    import sys
    import types
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "taiwan-whisper_amd"))
    import tw.distill as D
    _init(rank, world, port)
    calls = []
    D.F = types.SimpleNamespace(l2norm=lambda g, norm, ws: (calls.append(("norm", g.clone())), norm.fill_(float(g.norm()))),
                                adamw=lambda p32, g, m, v, p16, lr, b1, b2, eps, wd, t, norm, mx, inv_scale=1.0:
                                calls.append(("adamw", lr, t)))

    class Stub:
        pass
    st = D.DistillationTrainer.__new__(D.DistillationTrainer)
    st.s, st.bw = Stub(), Stub()
    st.s.grad = torch.full((5000,), float(rank + 1))
    st.s.store = Stub()
    st.s.store.p32 = st.s.store.p16 = torch.zeros(5000)
    st.m_buf, st.v_buf = torch.zeros(5000), torch.zeros(5000)
    st.world, st.pg, st.bucket, st.fold_world, st.dp = world, dist.group.WORLD, 1024, True, world > 1
    st.scaler = None
    st.norm, st.ws = torch.zeros(1), torch.zeros(8)
    st.runs = [(0, 5000, 0.0)]
    st.lr, st.warmup, st.sched, st.step = 1e-3, 0, "constant", 4
    st.b1 = st.b2 = st.eps = st.wd = 0.0
    st.max_grad_norm = 1.0
    st.overlap_update, st._update = True, None
    st._pending, st._reduced = [], []
    st.optimizer_step()
    assert calls == [] and st._update == (1e-3, 5) and st.step == 5 and len(st._pending) == 5
    st.flush()
    assert [c[0] for c in calls] == ["norm", "adamw"] and calls[1][1:] == (1e-3, 5)
    assert torch.equal(calls[0][1], torch.full((5000,), 3.0))     # the exchanged (summed) gradient
    st.flush()
    assert len(calls) == 2 and st._update is None
    out[rank] = True
    dist.destroy_process_group()


def test_deferred_update_control_flow():
    out = mp.Manager().dict()
    mp.spawn(_worker_deferred, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] and out[1]


def _worker_world4(rank, world, port, out):
    """World 4: the per-layer exchange is launched in backward order as each layer's
    gradients become final (last decoder layer first), the tail (embeddings + final LayerNorm, no layer hook)
    after the backward, each slice cut into buckets in address order; exchange_log records bytes and the
    tail flag per bucket; with overlap_update nothing is applied until flush(), which then sees the DDP mean."""
    import sys
    import types
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "taiwan-whisper_amd"))
    import tw.distill as D
    _init(rank, world, port)
    launched = []
    real_ar = dist.all_reduce

    def rec_ar(t, group=None, async_op=False):
        launched.append((t.data_ptr() - base[0]) // 4)
        return real_ar(t, group=group, async_op=async_op)
    D.torch.distributed.all_reduce = rec_ar
    calls = []
    D.F = types.SimpleNamespace(l2norm=lambda g, norm, ws: (calls.append(("norm", g.clone())), norm.fill_(float(g.norm()))),
                                adamw=lambda p32, g, m, v, p16, lr, b1, b2, eps, wd, t, norm, mx, inv_scale=1.0:
                                calls.append(("adamw", lr, t)))

    class Stub:
        pass
    # flat gradient layout of a 2-decoder-layer student: [layer0 | layer1 | embed_tokens + final LN] (sizes uneven)
    ranges = {"model.decoder.layers.0.": (0, 3000), "model.decoder.layers.1.": (3000, 7000)}
    n = 12_345
    st = D.DistillationTrainer.__new__(D.DistillationTrainer)
    st.s, st.bw = Stub(), Stub()
    g0 = torch.randn(n, generator=torch.Generator().manual_seed(rank))
    st.s.grad = g0 / world                        # power-of-two world: 1/world folded into the loss gradient
    base = [st.s.grad.data_ptr()]
    st.s.grad_range = lambda prefix: ranges.get(prefix)
    st.s.store = Stub()
    st.s.store.p32 = st.s.store.p16 = torch.zeros(n)
    st.m_buf, st.v_buf = torch.zeros(n), torch.zeros(n)
    st.world, st.pg, st.bucket, st.fold_world, st.dp = world, dist.group.WORLD, 2048, True, world > 1
    st.scaler = None
    st.norm, st.ws = torch.zeros(1), torch.zeros(8)
    st.runs = [(0, n, 0.0)]
    st.lr, st.warmup, st.sched, st.step = 1e-3, 0, "constant", 0
    st.b1 = st.b2 = st.eps = st.wd = 0.0
    st.max_grad_norm = 1.0
    st.overlap_update, st._update = True, None
    st.exchange_log, st.exchange_events = [], None
    st._pending, st._reduced = [], []
    st.bw.on_ready = st._grad_ready
    # the backward finishes the layers last-first and fires the hook per layer
    st.bw.on_ready("model.decoder.layers.1.")
    st.bw.on_ready("model.decoder.layers.0.")
    st.optimizer_step()                           # launches the tail, defers the update
    assert calls == [] and st._update == (1e-3, 1) and st.bw.on_ready is None
    assert launched == [3000, 5048, 0, 2048, 7000, 9048, 11096], launched
    assert [b for b, _ in st.exchange_log] == [4 * x for x in (2048, 1952, 2048, 952, 2048, 2048, 1249)]
    assert [t for _, t in st.exchange_log] == [False] * 4 + [True] * 3
    assert sum(b for b, _ in st.exchange_log) == 4 * n
    st.flush()
    assert [c[0] for c in calls] == ["norm", "adamw"] and calls[1][1:] == (1e-3, 1)
    out[rank] = calls[0][1]
    dist.destroy_process_group()


def test_world4_launch_order_and_deferred_update():
    world = 4
    out = mp.Manager().dict()
    mp.spawn(_worker_world4, args=(world, _free_port(), out), nprocs=world, join=True)
    n = 12_345
    g = [torch.randn(n, generator=torch.Generator().manual_seed(r)) for r in range(world)]
    mean = sum(x / world for x in g)
    for r in range(world):
        assert torch.equal(out[r], out[0])
        assert torch.allclose(out[r], mean, rtol=1e-6, atol=1e-7)
