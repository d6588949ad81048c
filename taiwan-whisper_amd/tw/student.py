"""Student initialisation — drop-in for `training/create_student_model.py` and
`utils/model_utils.py`.

  init_student_model_from_teacher  create_student_model.py:99-226
      config copy with overridden layer counts (:131-137); maximally spaced layer map
      linspace(0, L-1, n, int) with the last index forced (:139-154) or explicit
      --decoder_layers_numbers; non-layer weights + same-index layers first
      (load_state_dict(strict=False), :157-177), then mapped layers (:179-192); save as an HF
      directory (config.json, generation_config.json, model.safetensors; :198-202); smoke forward
      (:204-221).
  mix_language_embeddings          model_utils.py:4-14 (row := sum_i w_i row(lang_i), in the
      weight dtype, accumulated from 0).
The copy runs device-to-device on the flat parameter buffers.
"""
from __future__ import annotations

import copy
import json
import os

import numpy as np
import torch

from .config import WhisperConfig
from .modeling import WhisperForConditionalGeneration, is_pseudo

# Whisper multilingual language tokens (tokenizer vocab is not needed for the ids the reference uses)
LANG_IDS = {"en": 50259, "zh": 50260, "de": 50261, "es": 50262, "ru": 50263, "ko": 50264, "fr": 50265,
            "ja": 50266, "pt": 50267, "tr": 50268}


def layer_mapping(n_teacher: int, n_student: int, explicit=None):
    if explicit is not None:
        return [int(x) for x in explicit]
    m = np.linspace(0, n_teacher - 1, n_student, dtype=int)
    m[-1] = n_teacher - 1
    return [int(x) for x in m]


def _lang_id(tokenizer, lang):
    if tokenizer is not None:
        return tokenizer.convert_tokens_to_ids(f"<|{lang}|>")
    return LANG_IDS[lang]


def mix_language_embeddings(model: WhisperForConditionalGeneration, tokenizer=None, languages=("zh", "en"),
                            target_language="zh", weights=None):
    """In place on the model's embed_tokens (fp32 master and bf16 mirror kept consistent)."""
    if weights is None:
        weights = [1.0 / len(languages)] * len(languages)
    tgt = _lang_id(tokenizer, target_language)
    E = model.state_view("model.decoder.embed_tokens.weight")
    with torch.no_grad():
        new = torch.zeros(E.shape[1], dtype=E.dtype, device=E.device)
        for lang, w in zip(languages, weights):
            new += E[_lang_id(tokenizer, lang)] * w
        E[tgt] = new
    if model.store.p32 is not None:
        model.store.v16("model.decoder.embed_tokens.weight")[tgt].copy_(new.to(torch.bfloat16))
    return model


def _copy_layer(dst: WhisperForConditionalGeneration, src: WhisperForConditionalGeneration, side, j_src, j_dst):
    pre_s, pre_d = f"model.{side}.layers.{j_src}.", f"model.{side}.layers.{j_dst}."
    for n in src.store.order:
        if n.startswith(pre_s):
            dn = pre_d + n[len(pre_s):]
            if dst.store.p32 is not None:
                dst.store.v32(dn).copy_(src.store.v32(n) if src.store.p32 is not None else src.store.v16(n))
            dst.store.v16(dn).copy_(src.store.v16(n))


def student_from_teacher(teacher: WhisperForConditionalGeneration, encoder_layers=None, decoder_layers=2,
                         decoder_layers_numbers=None, dtype=torch.float32):
    if decoder_layers_numbers is not None and len(decoder_layers_numbers) != decoder_layers:
        raise ValueError(f"Got {len(decoder_layers_numbers)} layers number for {decoder_layers} decoder layers.")
    tc = teacher.config
    sc = WhisperConfig(**copy.deepcopy(tc.to_dict()))
    sc.update({"encoder_layers": encoder_layers if encoder_layers is not None else tc.encoder_layers,
               "decoder_layers": decoder_layers})
    enc_map = layer_mapping(tc.encoder_layers, sc.encoder_layers)
    dec_map = layer_mapping(tc.decoder_layers, decoder_layers, decoder_layers_numbers)
    st = WhisperForConditionalGeneration(sc, dtype=dtype, device=teacher.device)
    # non-layer tensors
    for n in st.store.order:
        if ".layers." in n:
            continue
        if st.store.p32 is not None:
            st.store.v32(n).copy_(teacher.store.v32(n) if teacher.store.p32 is not None else teacher.store.v16(n))
        st.store.v16(n).copy_(teacher.store.v16(n))
    # load_state_dict(strict=False): same-index layers
    for side, n in (("encoder", sc.encoder_layers), ("decoder", decoder_layers)):
        for j in range(min(n, getattr(tc, f"{side}_layers"))):
            _copy_layer(st, teacher, side, j, j)
    # mapped layers ({teacher: student}, last wins), encoder only when encoder_layers is given
    for side, mp, active in (("decoder", dec_map, True), ("encoder", enc_map, encoder_layers is not None)):
        if not active:
            continue
        tmap = {}
        for s_layer, t_layer in enumerate(mp):
            tmap[t_layer] = s_layer
        for t_layer in range(getattr(tc, f"{side}_layers")):
            if t_layer in tmap:
                _copy_layer(st, teacher, side, t_layer, tmap[t_layer])
    st._refresh_ln32()
    st.generation_config = dict(teacher.generation_config or {}, forced_decoder_ids=None)
    return st, enc_map, dec_map


def init_student_model_from_teacher(teacher_checkpoint, encoder_layers=None, decoder_layers=2,
                                    decoder_layers_numbers=None, save_dir=None, mix_lang_emb=False, device="cuda",
                                    tokenizer=None, smoke_forward=True):
    teacher = teacher_checkpoint if isinstance(teacher_checkpoint, WhisperForConditionalGeneration) else \
        WhisperForConditionalGeneration.from_pretrained(teacher_checkpoint, device=device)
    if mix_lang_emb:
        mix_language_embeddings(teacher, tokenizer, languages=["en", "zh"], target_language="zh", weights=[0.5, 0.5])
    student, _, _ = student_from_teacher(teacher, encoder_layers, decoder_layers, decoder_layers_numbers)
    if save_dir is not None:
        student.save_pretrained(save_dir)
        gc = dict(student.generation_config or {})
        gc.setdefault("decoder_start_token_id", student.config.decoder_start_token_id)
        with open(os.path.join(save_dir, "generation_config.json"), "w") as f:
            json.dump(gc, f, indent=2)
        if smoke_forward:   # :204-221 — reload and run one forward on np.ones(16000)
            st2 = WhisperForConditionalGeneration.from_pretrained(save_dir, device=device)
            from .feature_extraction import WhisperFeatureExtractor
            fe = WhisperFeatureExtractor(device=device)
            feats = fe(np.ones(16000))
            ids = torch.full((1, 1), st2.config.decoder_start_token_id, dtype=torch.long, device=device)
            st2(conv_input=feats.conv_input, decoder_input_ids=ids)
    return student
