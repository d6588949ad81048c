"""The persistent decoder-step kernel (tw_decoder_layers, csrc/decode_step.hip) against the per-launch decode
step it replaces (tw_gemv_* + tw_decode_attn per Linear / attention, the TW_DECODE_MEGA=0 path), bit for bit.

Both paths run the same device bodies (gemv_impl.h, decode_impl.h), so every output must be identical: the
logits of every step, the residual stream and every layer's self-attention cache, for batch 1 / 3 / 8 (the
GEMV row blocks MR = 1 / 4 / 8), bf16 and fp16 models at whisper-large-v2 dims (d 1280, 20 heads, ffn 5120,
1500 encoder frames -> 12 key chunks of the split cross-attention), eager launches and HIP-graph replay.
The greedy / long-form token tests (tests/test_fp16_gpu.py, test_decode_configs_gpu.py c5, ...) run on the
persistent kernel by default as well (it is the path for every batch <= 8 bf16 / fp16 decode).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


_MODELS = {}


def _model(dtype):
    if dtype not in _MODELS:
        from tw.config import MODEL_DIMS, WhisperConfig
        from tw.modeling import WhisperForConditionalGeneration, random_init_
        cfg = WhisperConfig(**MODEL_DIMS["large-v2"])
        _MODELS.clear()
        _MODELS[dtype] = random_init_(WhisperForConditionalGeneration(cfg, dtype=dtype, device=DEV), seed=3)
    return _MODELS[dtype]


def _run(m, mega, enc16, ids, B, T_max, graph):
    from tw import generation as G
    old = G.MEGA
    G.MEGA = mega
    try:
        sess = G.DecodeSession(m, enc16, B, 1500, T_max)
    finally:
        G.MEGA = old
    assert sess.mega == mega
    sess.t_dev.zero_()
    logits = []
    for t in range(ids.shape[1]):
        sess.cur.copy_(ids[:, t])
        if graph and t >= 2:               # eager prefix, then one captured step replayed
            if sess.graph is None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    sess.step()
                sess.graph = g
            sess.graph.replay()
        else:
            sess.step()
        logits.append(sess.logits.clone())
    torch.cuda.synchronize()
    sess.check()
    return torch.stack(logits), sess.x.clone(), [c[:, :ids.shape[1]].clone() for c in sess.self_kv]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B", [1, 3, 8])
def test_decoder_step_kernel_bit_identical(dtype, B):
    m = _model(dtype)
    d = m.config.d_model
    g = torch.Generator(device="cpu").manual_seed(B)
    enc16 = (torch.randn(B * 1500, d, generator=g) * 0.5).to(DEV, dtype)
    ids = torch.randint(0, 50000, (B, 6), generator=g).to(DEV)
    T_max = 16
    ref = _run(m, False, enc16, ids, B, T_max, graph=False)
    for graph in (False, True):
        got = _run(m, True, enc16, ids, B, T_max, graph=graph)
        assert torch.isfinite(ref[0].float()).all()
        assert torch.equal(got[0], ref[0]), f"logits differ (graph={graph})"
        assert torch.equal(got[1], ref[1]), "residual stream differs"
        for i, (a, b) in enumerate(zip(got[2], ref[2])):
            assert torch.equal(a, b), f"self-attention cache of layer {i} differs"


def test_decoder_step_kernel_greedy_ids_match():
    """generate() end to end (prompt prefill, captured step graph, selection): ids identical with and without
    the persistent kernel, batch 2, fp16 (the reference's run_eval.py:99 default dtype)."""
    from tw import generation as G
    from tw.config import LARGE_V2_SUPPRESS, GenerationConfig
    m = _model(torch.float16)
    m.generation_config = GenerationConfig(suppress_tokens=LARGE_V2_SUPPRESS, begin_suppress_tokens=[220, 50257],
                                           lang_to_id={"<|zh|>": 50260}, max_initial_timestamp_index=50)
    g = torch.Generator(device="cpu").manual_seed(11)
    mel = (torch.randn(2, 80, 3000, generator=g) * 0.3).to(DEV)
    outs = []
    for mega in (False, True):
        old = G.MEGA
        G.MEGA = mega
        try:
            outs.append(m.generate(mel, language="zh", task="transcribe", max_new_tokens=24).cpu())
        finally:
            G.MEGA = old
    assert outs[0].shape == outs[1].shape and torch.equal(outs[0], outs[1])
