"""torch.ops.tw.* on the GPU (tw/torch_ops.py).

* A whole decoder stack (embedding -> per layer: LN, fused QKV, causal self-attention, out_proj + residual, LN,
  cross-q, cross-KV, cross-attention, out_proj + residual, LN, fc1 + GELU, fc2 + residual -> final LN) composed
  from the torch operators is BIT-IDENTICAL to the engine's own ctypes path (WhisperForConditionalGeneration.decode)
  on the micro config, bf16 model: the operators run the same kernels with the same arguments.
* Autograd through the operators (register_autograd -> the HIP backward kernels) against an fp32 torch autograd
  reference of the same layer: cosine >= 0.999 and relative L2 <= max(3e-2, 2 x the distance of the same layer
  under torch bf16 autocast -- the reference's own arithmetic -- to fp32) per gradient.
* torch.library.opcheck: schema, autograd registration and fake-tensor consistency of every trainable op.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    # the operators register on import of tw.torch_ops; a test selection that runs only this module's opcheck
    # cases must not depend on another test having imported it first
    import tw.torch_ops  # noqa: F401


def _v3(t, B, T, off, C):
    """[B*T, ld] matrix -> [B, T, C] view of columns off..off+C (strided rows)."""
    ld = t.stride(0)
    return torch.as_strided(t, (B, T, C), (T * ld, ld, 1), t.storage_offset() + off)


def _layer_ops(m, x, enc16, p, B, T, Tk):
    """One decoder layer from torch.ops.tw.* (the arithmetic of tw.modeling _attn/_cross/_mlp_block)."""
    tw = torch.ops.tw
    d = m.config.d_model
    M = B * T
    a = p + ".self_attn"
    y = tw.layer_norm(x, m.ln_param(a + "_layer_norm.weight"), m.ln_param(a + "_layer_norm.bias"), 1e-5)[0]
    qkv = tw.linear(y, m.wspan(a + ".q_proj.weight", a + ".v_proj.weight", (3 * d, d)),
                    m.wspan(a + ".q_proj.bias", a + ".v_proj.bias", (3 * d,)))
    o = tw.attention(_v3(qkv, B, T, 0, d), _v3(qkv, B, T, d, d), _v3(qkv, B, T, 2 * d, d), True, 0.125)[0]
    x = tw.linear_residual(o.view(M, d), m._w16(a + ".out_proj.weight"), m._w16(a + ".out_proj.bias"), x)
    c = p + ".encoder_attn"
    y = tw.layer_norm(x, m.ln_param(c + "_layer_norm.weight"), m.ln_param(c + "_layer_norm.bias"), 1e-5)[0]
    q = tw.linear(y, m._w16(c + ".q_proj.weight"), m._w16(c + ".q_proj.bias"))
    kv = tw.linear(enc16, m.wspan(c + ".k_proj.weight", c + ".v_proj.weight", (2 * d, d)),
                   m.wspan(c + ".k_proj.zero_bias", c + ".v_proj.bias", (2 * d,)))
    o = tw.attention(q.view(B, T, d), _v3(kv, B, Tk, 0, d), _v3(kv, B, Tk, d, d), False, 0.125)[0]
    x = tw.linear_residual(o.view(M, d), m._w16(c + ".out_proj.weight"), m._w16(c + ".out_proj.bias"), x)
    y = tw.layer_norm(x, m.ln_param(p + ".final_layer_norm.weight"), m.ln_param(p + ".final_layer_norm.bias"),
                      1e-5)[0]
    h, _ = tw.linear_gelu(y, m._w16(p + ".fc1.weight"), m._w16(p + ".fc1.bias"))
    return tw.linear_residual(h, m._w16(p + ".fc2.weight"), m._w16(p + ".fc2.bias"), x)


def _micro_bf16():
    from test_decode_gpu import _micro
    cfg, w, m, _ = _micro(dtype=torch.bfloat16)
    return cfg, m


def test_decoder_stack_bit_identical_to_ctypes_path():
    cfg, m = _micro_bf16()
    B, T, Tk = 3, 37, 1500
    g = torch.Generator(device=DEV).manual_seed(7)
    ids = torch.randint(0, 51865, (B, T), device=DEV, generator=g)
    enc16 = (torch.randn(B * Tk, cfg["d_model"], device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    want = m.decode(ids, enc16, Tk)
    x = m.embed(ids)
    for i in range(cfg["decoder_layers"]):
        x = _layer_ops(m, x, enc16, f"model.decoder.layers.{i}", B, T, Tk)
    got = torch.ops.tw.layer_norm(x, m.ln_param("model.decoder.layer_norm.weight"),
                                  m.ln_param("model.decoder.layer_norm.bias"), 1e-5)[0]
    torch.cuda.synchronize()
    assert got.dtype == want.dtype and got.shape == want.shape
    assert torch.equal(got, want)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _cos(a, b):
    return float(torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0))


def test_layer_autograd_vs_fp32_torch():
    """Gradients of a decoder layer's parameters and of its input stream through torch.ops.tw (HIP backward
    kernels) vs the same layer in fp32 torch autograd."""
    cfg, m = _micro_bf16()
    d, f = cfg["d_model"], cfg["decoder_ffn_dim"]
    B, T, Tk = 2, 29, 1500
    g = torch.Generator(device=DEV).manual_seed(3)
    p = "model.decoder.layers.0"
    names = {"ln1": "self_attn_layer_norm", "ln2": "encoder_attn_layer_norm", "ln3": "final_layer_norm"}
    W = {
        "wqkv": m.wspan(p + ".self_attn.q_proj.weight", p + ".self_attn.v_proj.weight", (3 * d, d)),
        "bqkv": m.wspan(p + ".self_attn.q_proj.bias", p + ".self_attn.v_proj.bias", (3 * d,)),
        "wo": m._w16(p + ".self_attn.out_proj.weight"), "bo": m._w16(p + ".self_attn.out_proj.bias"),
        "wq": m._w16(p + ".encoder_attn.q_proj.weight"), "bq": m._w16(p + ".encoder_attn.q_proj.bias"),
        "wkv": m.wspan(p + ".encoder_attn.k_proj.weight", p + ".encoder_attn.v_proj.weight", (2 * d, d)),
        "wco": m._w16(p + ".encoder_attn.out_proj.weight"), "bco": m._w16(p + ".encoder_attn.out_proj.bias"),
        "w1": m._w16(p + ".fc1.weight"), "b1": m._w16(p + ".fc1.bias"),
        "w2": m._w16(p + ".fc2.weight"), "b2": m._w16(p + ".fc2.bias"),
    }
    for k, nm in names.items():
        W[k + "w"] = m.ln_param(f"{p}.{nm}.weight") + 0.1 * torch.randn(d, device=DEV, generator=g)
        W[k + "b"] = m.ln_param(f"{p}.{nm}.bias") + 0.1 * torch.randn(d, device=DEV, generator=g)
    P16 = {k: v.detach().clone().requires_grad_(True) for k, v in W.items()}
    P32 = {k: v.detach().float().clone().requires_grad_(True) for k, v in W.items()}
    x0 = torch.randn(B * T, d, device=DEV, generator=g)
    enc = (torch.randn(B * Tk, d, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    G = torch.randn(B * T, d, device=DEV, generator=g)

    def run_tw(P, x):
        tw = torch.ops.tw
        y = tw.layer_norm(x, P["ln1w"], P["ln1b"], 1e-5)[0]
        qkv = tw.linear(y, P["wqkv"], P["bqkv"])
        q, k, v = (qkv[:, i * d:(i + 1) * d].reshape(B, T, d) for i in range(3))
        o = tw.attention(q, k, v, True, 0.125)[0]
        x = tw.linear_residual(o.reshape(B * T, d), P["wo"], P["bo"], x)
        y = tw.layer_norm(x, P["ln2w"], P["ln2b"], 1e-5)[0]
        q = tw.linear(y, P["wq"], P["bq"])
        kv = tw.linear(enc, P["wkv"], None)
        o = tw.attention(q.view(B, T, d), kv[:, :d].reshape(B, Tk, d), kv[:, d:].reshape(B, Tk, d), False, 0.125)[0]
        x = tw.linear_residual(o.reshape(B * T, d), P["wco"], P["bco"], x)
        y = tw.layer_norm(x, P["ln3w"], P["ln3b"], 1e-5)[0]
        h, _ = tw.linear_gelu(y, P["w1"], P["b1"])
        return tw.linear_residual(h, P["w2"], P["b2"], x)

    def run_ref(P, x):
        import torch.nn.functional as Fn
        H = d // 64

        def att(q, k, v, causal):
            sh = lambda t: t.view(B, -1, H, 64).transpose(1, 2)
            o = Fn.scaled_dot_product_attention(sh(q), sh(k), sh(v), is_causal=causal, scale=0.125)
            return o.transpose(1, 2).reshape(-1, d)
        y = Fn.layer_norm(x, (d,), P["ln1w"], P["ln1b"], 1e-5)
        qkv = y @ P["wqkv"].T + P["bqkv"]
        x = x + att(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], True) @ P["wo"].T + P["bo"]
        y = Fn.layer_norm(x, (d,), P["ln2w"], P["ln2b"], 1e-5)
        q = y @ P["wq"].T + P["bq"]
        kv = enc.float() @ P["wkv"].T
        x = x + att(q, kv[:, :d], kv[:, d:], False) @ P["wco"].T + P["bco"]
        y = Fn.layer_norm(x, (d,), P["ln3w"], P["ln3b"], 1e-5)
        h = Fn.gelu(y @ P["w1"].T + P["b1"])
        return x + h @ P["w2"].T + P["b2"]

    x16 = x0.clone().requires_grad_(True)
    x32 = x0.clone().requires_grad_(True)
    out16 = run_tw(P16, x16)
    out32 = run_ref(P32, x32)
    assert out16.dtype == torch.float32                     # the fp32 stream stays fp32 through the residual ops
    assert _rel(out16, out32) < 1e-2
    (out16 * G).sum().backward()
    (out32 * G).sum().backward()
    # the reference's own arithmetic: the same fp32 layer under torch bf16 autocast (run_distillation.py runs the
    # student under Accelerator(mixed_precision="bf16")); its distance to fp32 is the noise floor a bf16 backward has
    PA = {k: v.detach().float().clone().requires_grad_(True) for k, v in W.items()}
    xa = x0.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        outa = run_ref(PA, xa)
    (outa.float() * G).sum().backward()
    torch.cuda.synchronize()
    pairs = [("x", x16.grad, x32.grad, xa.grad)] + [(k, P16[k].grad, P32[k].grad, PA[k].grad) for k in P16]
    for k, a, b, c in pairs:
        assert a is not None, k
        # 3e-2, or twice the autocast reference's own distance to fp32 where that is larger (the LayerNorm weights:
        # sums over rows of bf16-rounded products; the round-4 bound of 6e-2 for them is replaced by this measure)
        bound = max(3e-2, 2 * _rel(c, b))
        assert _rel(a, b) <= bound and _cos(a, b) >= 0.999, (k, _rel(a, b), _cos(a, b), "autocast ref", _rel(c, b))


def test_kl_ce_op_gradient_is_the_fused_kernel():
    """tw::kl_ce: the loss triple of the fused kernel, and autograd hands back its dlogits (x the loss grad)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    rows, Vp, V = 40, 51904, 51865
    s = (torch.randn(rows, Vp, device=DEV, generator=g) * 3).to(torch.bfloat16)
    s[:, V:] = 0
    t = (torch.randn(rows, Vp, device=DEV, generator=g) * 3).to(torch.bfloat16)
    t[:, V:] = 0
    lab = torch.randint(0, V, (rows,), device=DEV, generator=g)
    lab[::7] = -100
    s_leaf = s.clone().requires_grad_(True)
    out3, dl = torch.ops.tw.kl_ce(s_leaf, t, lab, V, 2.0, 0.8, 1.0)
    out3[0].backward()
    torch.cuda.synchronize()
    assert torch.equal(s_leaf.grad, dl)
    # CE part against torch (fp32 log-softmax over the real vocabulary, mean over valid labels)
    ce = torch.nn.functional.cross_entropy(s[:, :V].float(), lab, ignore_index=-100)
    assert abs(float(out3[1]) - float(ce)) <= 1e-4 * abs(float(ce))


def test_log_mel_op_matches_feature_extractor():
    from tw.feature_extraction import WhisperFeatureExtractor
    from tw.data import synthetic_audio
    wav = synthetic_audio(2, seed=3, device=torch.device(DEV))
    mel = torch.ops.tw.log_mel(wav)
    ref, _ = WhisperFeatureExtractor(device=torch.device(DEV)).extract(wav, want_conv_input=False)
    torch.cuda.synchronize()
    assert torch.equal(mel, ref)


def test_fp16_backward_raises_not_implemented():
    """The fp16 model is forward-only: every trainable op's backward raises NotImplementedError."""
    g = torch.Generator(device=DEV).manual_seed(2)
    x = (torch.randn(64, 128, device=DEV, generator=g) * 0.3).half().requires_grad_(True)
    w = (torch.randn(256, 128, device=DEV, generator=g) * 0.3).half().requires_grad_(True)
    for op in (lambda: torch.ops.tw.linear_gelu(x, w, None)[0], lambda: torch.ops.tw.linear(x, w, None)):
        y = op()
        with pytest.raises(NotImplementedError):
            y.float().sum().backward()


@pytest.mark.parametrize("op", ["linear", "linear_gelu", "linear_residual", "layer_norm", "attention"])
def test_opcheck(op):
    g = torch.Generator(device=DEV).manual_seed(1)
    r = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.3).to(torch.bfloat16)
    x, w, b = r(64, 128), r(256, 128), r(256)
    args = {
        "linear": (x, w, b),
        "linear_gelu": (x, w, b),
        "linear_residual": (x, w, b, torch.randn(64, 256, device=DEV, generator=g)),
        "layer_norm": (torch.randn(64, 128, device=DEV, generator=g), torch.ones(128, device=DEV),
                       torch.zeros(128, device=DEV), 1e-5),
        "attention": (r(2, 40, 128), r(2, 50, 128), r(2, 50, 128), False, 0.125),
    }[op]
    torch.library.opcheck(getattr(torch.ops.tw, op).default, args,
                          test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))
