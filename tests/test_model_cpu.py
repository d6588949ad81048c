"""Host-side model logic without a GPU: engine layout <-> HF state-dict round trip, fused
views, trainable packing, safetensors I/O format."""
import numpy as np
import torch

from oracle.weights import CONFIGS, make_weights


def _model(dtype=torch.float32):
    from tw.config import WhisperConfig
    from tw.modeling import WhisperForConditionalGeneration
    cfg = CONFIGS["micro"]
    w = make_weights(cfg, 3)
    m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg), {k: torch.from_numpy(v) for k, v in
                                                                              w.items()}, dtype=dtype, device="cpu")
    return cfg, w, m


def test_state_dict_roundtrip_and_layout():
    cfg, w, m = _model()
    sd = m.state_dict()
    assert set(sd) == set(w) | {"proj_out.weight"}
    for k, v in w.items():
        assert tuple(sd[k].shape) == v.shape, k
        np.testing.assert_array_equal(sd[k].numpy(), v)
    d = cfg["d_model"]
    # fused QKV view == cat(q, k, v); k has a zero bias segment
    p = "model.encoder.layers.1.self_attn"
    fused = m.store.span(m.store.p32, p + ".q_proj.weight", p + ".v_proj.weight", (3 * d, d))
    np.testing.assert_array_equal(fused.numpy(), np.concatenate([w[p + ".q_proj.weight"], w[p + ".k_proj.weight"],
                                                                 w[p + ".v_proj.weight"]]))
    bias = m.store.span(m.store.p32, p + ".q_proj.bias", p + ".v_proj.bias", (3 * d,)).numpy()
    assert (bias[d:2 * d] == 0).all()
    # conv weight engine layout [d][tap][c]
    c1 = m.store.v32("model.encoder.conv1.weight").view(d, 3, 80)
    np.testing.assert_array_equal(c1.numpy(), w["model.encoder.conv1.weight"].transpose(0, 2, 1))
    # vocab padded with zero rows
    E = m.store.v32("model.decoder.embed_tokens.weight")
    assert E.shape[0] == 51904 and (E[51865:] == 0).all()
    # bf16 mirror
    assert torch.equal(m.store.v16(p + ".q_proj.weight"), m.store.v32(p + ".q_proj.weight").bfloat16())


def test_pack_for_training_keeps_values_and_spans():
    cfg, w, m = _model()
    m.set_trainable("", True)
    m.set_trainable("model.encoder", False)
    m.set_trainable("model.decoder.embed_positions", False)
    m.pack_for_training()
    assert m.grad.numel() == m.train_prefix
    assert all(m.store.offset[n] < m.train_prefix for n in m.train_names)
    for k, v in w.items():
        np.testing.assert_array_equal(m.state_dict()[k].numpy(), v)
    assert m.gv("model.encoder.layers.0.fc1.weight") is None
    assert m.gv("model.decoder.layers.0.fc1.weight").shape == (cfg["decoder_ffn_dim"], cfg["d_model"])
    p = "model.decoder.layers.1.encoder_attn"
    m.store.span(m.grad, p + ".k_proj.weight", p + ".v_proj.weight", (2 * cfg["d_model"], cfg["d_model"]))


def test_save_load_pretrained(tmp_path):
    from tw.modeling import WhisperForConditionalGeneration
    cfg, w, m = _model()
    m.save_pretrained(tmp_path)
    from safetensors.numpy import load_file
    sd = load_file(str(tmp_path / "model.safetensors"))
    assert set(sd) == set(w)
    m2 = WhisperForConditionalGeneration.from_pretrained(str(tmp_path), device="cpu")
    for k in w:
        np.testing.assert_array_equal(m2.state_dict()[k].numpy(), w[k])
    mb = WhisperForConditionalGeneration.from_pretrained(str(tmp_path), torch_dtype=torch.bfloat16, device="cpu")
    assert mb.store.p32 is None
    assert torch.equal(mb.ln_param("model.decoder.layer_norm.weight"),
                       torch.from_numpy(w["model.decoder.layer_norm.weight"]).bfloat16().float())
