"""Product student creation (tw/student.py) against the reference's own functions.

The fixtures in tests/golden/student.npz were produced by importing the reference's
`init_student_model_from_teacher` (training/create_student_model.py:99-226) and
`mix_language_embeddings` (utils/model_utils.py:4-14) in the build container
(tests/golden/make_golden.py gen_student).  Here the PRODUCT path runs on CPU tensors
(the flat parameter store is plain torch memory; no kernel is launched) and must reproduce
every saved tensor bit for bit (per-key float64 checksums of identical arrays are identical).
"""
import json
import os

import numpy as np
import pytest
import torch
from safetensors.numpy import load_file

from conftest import load_golden
from oracle.weights import CONFIGS, SPECIAL, make_weights
from tw.config import WhisperConfig
from tw.modeling import WhisperForConditionalGeneration
from tw.student import init_student_model_from_teacher, layer_mapping, mix_language_embeddings, student_from_teacher

CFG = dict(CONFIGS["micro"], encoder_layers=4, decoder_layers=5)
CASES = {"e2_d2": dict(encoder_layers=2, decoder_layers=2), "d3": dict(decoder_layers=3),
         "e3_dnums": dict(encoder_layers=3, decoder_layers=2, decoder_layers_numbers=[1, 4]),
         "mix": dict(encoder_layers=2, decoder_layers=2, mix_lang_emb=True)}


def _teacher(dtype=torch.float32):
    w = make_weights(CFG, 7)
    return WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**CFG), {k: torch.from_numpy(v)
                                                                                 for k, v in w.items()},
                                                           dtype=dtype, device="cpu")


def _checksums(sd):
    return {k: float(np.asarray(v, np.float64).sum()) for k, v in sd.items()}


@pytest.fixture(scope="module")
def teacher_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("teacher"))
    t = _teacher()
    t.generation_config = {"decoder_start_token_id": SPECIAL["sot"]}
    t.save_pretrained(d)
    return d


@pytest.mark.parametrize("name", list(CASES))
def test_init_student_model_from_teacher_matches_reference(name, teacher_dir, tmp_path):
    """init_student_model_from_teacher(save_dir=...) writes the reference's student: same config layer
    counts, same key set, every tensor identical (incl. mix_lang_emb on the fp32 teacher)."""
    g = load_golden("student")
    meta = json.loads(str(g["student_meta"]))[name]
    out = str(tmp_path / name)
    init_student_model_from_teacher(teacher_dir, save_dir=out, device="cpu", smoke_forward=False, **CASES[name])
    cfg = json.load(open(os.path.join(out, "config.json")))
    assert (cfg["encoder_layers"], cfg["decoder_layers"]) == (meta["encoder_layers"], meta["decoder_layers"])
    sd = load_file(os.path.join(out, "model.safetensors"))
    assert sorted(sd) == meta["keys"]
    for k, v in _checksums(sd).items():
        assert v == float(g[f"{name}|{k}"]), (name, k, v, float(g[f"{name}|{k}"]))
    gc = json.load(open(os.path.join(out, "generation_config.json")))
    assert gc.get("forced_decoder_ids") is None and gc["decoder_start_token_id"] == SPECIAL["sot"]


def test_student_from_teacher_in_memory_views():
    """student_from_teacher on the flat store: layer map and HF-keyed views (engine layout undone)."""
    t = _teacher()
    st, enc_map, dec_map = student_from_teacher(t, encoder_layers=3, decoder_layers=2, decoder_layers_numbers=[1, 4])
    assert enc_map == layer_mapping(4, 3) == [0, 1, 3] and dec_map == [1, 4]
    tsd, ssd = t.state_dict(), st.state_dict()
    for j_s, j_t in enumerate(dec_map):
        for suffix in ("self_attn.k_proj.weight", "encoder_attn.v_proj.bias", "fc1.weight", "final_layer_norm.bias"):
            torch.testing.assert_close(ssd[f"model.decoder.layers.{j_s}.{suffix}"],
                                       tsd[f"model.decoder.layers.{j_t}.{suffix}"], rtol=0, atol=0)
    torch.testing.assert_close(ssd["model.encoder.conv1.weight"], tsd["model.encoder.conv1.weight"], rtol=0, atol=0)
    # bf16 mirror is the cast of the fp32 master for every copied tensor
    assert torch.equal(st.store.p16, st.store.p32.to(torch.bfloat16))
    with pytest.raises(ValueError):
        student_from_teacher(t, decoder_layers=2, decoder_layers_numbers=[0])


def test_mix_language_embeddings_bf16_teacher_bit_exact():
    """The training entry point mixes the bf16 teacher (run_distillation.py:1019-1020, languages zh,en):
    row arithmetic in bf16, bit-identical to the reference function's row."""
    g = load_golden("student")
    t = _teacher(torch.bfloat16)
    mix_language_embeddings(t, None, languages=["zh", "en"])
    row = t.state_view("model.decoder.embed_tokens.weight")[SPECIAL["zh"]]
    assert row.dtype == torch.bfloat16
    np.testing.assert_array_equal(row.view(torch.int16).numpy(), g["mix_bf16_row_u16"])


def test_mix_language_embeddings_f32_master_and_mirror():
    """fp32-master model: the fp32 row equals the reference's fp32 row and the bf16 mirror is its cast."""
    g = load_golden("student")
    t = _teacher()
    before = t.state_view("model.decoder.embed_tokens.weight").clone()
    mix_language_embeddings(t, None, languages=["en", "zh"], weights=[0.5, 0.5])
    E = t.state_view("model.decoder.embed_tokens.weight")
    np.testing.assert_array_equal(E[SPECIAL["zh"]].numpy(), g["mix_f32_row"])
    assert torch.equal(t.store.v16("model.decoder.embed_tokens.weight")[SPECIAL["zh"]],
                       E[SPECIAL["zh"]].to(torch.bfloat16))
    other = torch.ones(E.shape[0], dtype=torch.bool)
    other[SPECIAL["zh"]] = False
    assert torch.equal(E[other], before[other])


def test_run_distillation_mixes_teacher_only(tmp_path):
    """--mix_lang_emb mixes the teacher only (run_distillation.py:1019-1020); the student row was mixed
    once at creation (create_student_model.py:124-125) and is loaded unchanged."""
    import argparse
    from tw.run_distillation import load_models
    t = _teacher(torch.bfloat16)
    t.save_pretrained(str(tmp_path / "t"))
    st, _, _ = student_from_teacher(_teacher(), encoder_layers=2, decoder_layers=2)
    mix_language_embeddings(st, None, languages=["en", "zh"], weights=[0.5, 0.5])
    st.save_pretrained(str(tmp_path / "s"))
    args = argparse.Namespace(teacher_model_name_or_path=str(tmp_path / "t"), model_name_or_path=str(tmp_path / "s"),
                              dtype="bfloat16", mix_lang_emb=True)
    teacher, student = load_models(args, "cpu")
    g = load_golden("student")
    np.testing.assert_array_equal(teacher.state_view("model.decoder.embed_tokens.weight")[SPECIAL["zh"]]
                                  .view(torch.int16).numpy(), g["mix_bf16_row_u16"])
    np.testing.assert_array_equal(student.state_view("model.decoder.embed_tokens.weight")[SPECIAL["zh"]].numpy(),
                                  st.state_view("model.decoder.embed_tokens.weight")[SPECIAL["zh"]].numpy())
    args.dtype = "float16"          # mixed_precision="fp16": fp16 teacher, fp32-master student under fp16 autocast
    teacher, student = load_models(args, "cpu")
    assert teacher.dtype == torch.float16 and teacher.compute == "fp16"
    assert student.dtype == torch.float32 and student.compute == "fp16" and student.store.p16.dtype == torch.float16
