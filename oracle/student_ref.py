"""ORACLE (test infrastructure only): student initialisation restatement.

* `layer_mapping` restates `training/create_student_model.py:139-154`:
  np.linspace(0, L_teacher - 1, L_student, dtype=int) with the last index forced to
  L_teacher - 1 (or the explicit --decoder_layers_numbers).
* `init_student_from_teacher` restates `:131-192` on an HF-keyed state dict: copy
  every non-layer tensor, then student layer j := teacher layer map[j].
* `mix_language_embeddings` restates `utils/model_utils.py:4-14`: the target
  language row := 0 + sum_i w_i * row(lang_i), accumulated in the weight dtype.
"""
from __future__ import annotations

import copy

import numpy as np


def layer_mapping(n_teacher: int, n_student: int, explicit=None):
    if explicit is not None:
        return list(explicit)
    m = np.linspace(0, n_teacher - 1, n_student, dtype=int)
    m[-1] = n_teacher - 1
    return [int(x) for x in m]


def init_student_from_teacher(teacher_cfg: dict, teacher_sd: dict, encoder_layers=None,
                              decoder_layers=2, decoder_layers_numbers=None):
    cfg = copy.deepcopy(teacher_cfg)
    cfg["encoder_layers"] = encoder_layers if encoder_layers is not None else teacher_cfg["encoder_layers"]
    cfg["decoder_layers"] = decoder_layers
    enc_map = layer_mapping(teacher_cfg["encoder_layers"], cfg["encoder_layers"])
    dec_map = layer_mapping(teacher_cfg["decoder_layers"], decoder_layers, decoder_layers_numbers)
    sd = {}
    for k, v in teacher_sd.items():
        if ".layers." not in k:
            sd[k] = v.copy()
    # reference: load_state_dict(teacher, strict=False) fills student layers 0..n-1 from
    # teacher layers 0..n-1 first, then overwrites mapped layers (:157-192)
    def copy_layer(side, src, dst):
        pre_t, pre_s = f"model.{side}.layers.{src}.", f"model.{side}.layers.{dst}."
        for k, v in teacher_sd.items():
            if k.startswith(pre_t):
                sd[pre_s + k[len(pre_t):]] = v.copy()

    for side, n in (("encoder", cfg["encoder_layers"]), ("decoder", decoder_layers)):
        for j in range(min(n, teacher_cfg[f"{side}_layers"])):   # strict=False load, same index
            copy_layer(side, j, j)
    for side, mp, active in (("decoder", dec_map, True), ("encoder", enc_map, encoder_layers is not None)):
        if not active:
            continue
        tmap = {}
        for s_layer, t_layer in enumerate(mp):                  # {teacher: student}, last wins
            tmap[t_layer] = s_layer
        for t_layer in range(teacher_cfg[f"{side}_layers"]):
            if t_layer in tmap:
                copy_layer(side, t_layer, tmap[t_layer])
    return cfg, sd, enc_map, dec_map


def mix_language_embeddings(embed: np.ndarray, lang_ids, target_id, weights=None):
    """In-place on a [V, d] array (float32 or bf16-as-uint16 handled by caller)."""
    if weights is None:
        weights = [1.0 / len(lang_ids)] * len(lang_ids)
    new = np.zeros(embed.shape[1], dtype=embed.dtype)
    for lid, w in zip(lang_ids, weights):
        new = (new + embed[lid] * embed.dtype.type(w)).astype(embed.dtype)
    embed[target_id] = new
    return embed
