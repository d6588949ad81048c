"""ORACLE (test infrastructure only): the deterministic INPUTS and settings of the golden fixtures -- features,
label batches, weight recipes and generation settings as plain data -- shared by the fixture generator
(tests/golden/make_golden.py, build container, HF Transformers) and the GPU parity tests (which must not import the
generator or HF Transformers: VERDICT r05 item 8).  Nothing here imports transformers.

Generation settings are plain dicts with the field names of HF `GenerationConfig` (make_golden builds the HF object
from them; the tests build tw.config.GenerationConfig).
"""
from __future__ import annotations

import numpy as np

from . import labels as L
from . import logmel
from .weights import CONFIGS, SPECIAL, make_weights

# large-v2 generation_config.suppress_tokens (test parameter for the suppress processor)
SUPPRESS = [1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93,
            359, 503, 522, 542, 873, 893, 902, 918, 922, 931, 1350, 1853, 1982, 2460, 2627, 3246,
            3253, 3268, 3536, 3846, 3961, 4183, 4667, 6585, 6647, 7273, 9061, 9383, 10428, 10929,
            11938, 12033, 12331, 12562, 13793, 14157, 14635, 15265, 15618, 16553, 16604, 18362,
            18956, 20075, 21675, 22520, 26130, 26161, 26435, 28279, 29464, 31650, 32302, 32470,
            36865, 42863, 47425, 49870, 50254, 50258, 50358, 50359, 50360, 50361, 50362]
ROWS = [0, 3, 4, 57, 200, 446]          # decoder positions whose full logit rows are checked
VSTRIDE = 97                             # vocab subsample stride for stored logit rows

# timestamp / long-form generation settings (the large-v2 checkpoint's generation_config fields the path reads)
TS_GENERATION = dict(decoder_start_token_id=SPECIAL["sot"], eos_token_id=SPECIAL["eot"], pad_token_id=SPECIAL["pad"],
                     bos_token_id=SPECIAL["eot"], suppress_tokens=SUPPRESS,
                     begin_suppress_tokens=[220, SPECIAL["eot"]], max_length=448, num_beams=1, do_sample=False,
                     no_timestamps_token_id=SPECIAL["notimestamps"], is_multilingual=True,
                     lang_to_id={"<|en|>": SPECIAL["en"], "<|zh|>": SPECIAL["zh"]},
                     task_to_id={"transcribe": SPECIAL["transcribe"], "translate": 50358},
                     max_initial_timestamp_index=50)
# greedy without timestamps at large-v2 dims (decoder_input_ids prompt).  The timestamp tokens are suppressed too:
# with random weights a row can emit a timestamp pair after <|notimestamps|>, after which HF's seek loop decodes a
# second window for that row even without return_timestamps -- a path the engine's decoder_input_ids decode does not
# take and a trained checkpoint does not reach
LV2_GREEDY_SUPPRESS = SUPPRESS + list(range(SPECIAL["timestamp_begin"], 51865))
LV2_GREEDY_GENERATION = dict(decoder_start_token_id=SPECIAL["sot"], eos_token_id=SPECIAL["eot"],
                             pad_token_id=SPECIAL["pad"], suppress_tokens=LV2_GREEDY_SUPPRESS,
                             begin_suppress_tokens=[220, SPECIAL["eot"]], max_length=448, num_beams=1,
                             do_sample=False, no_timestamps_token_id=SPECIAL["notimestamps"])
TW_GENERATION_KEYS = ("decoder_start_token_id", "eos_token_id", "pad_token_id", "suppress_tokens",
                      "begin_suppress_tokens", "max_length", "no_timestamps_token_id", "is_multilingual", "lang_to_id",
                      "task_to_id", "max_initial_timestamp_index")


def longform_features():
    """Deterministic synthetic log-mel-range features for the long-form fixture (80 x 6500 frames =
    65 s; feature extraction is pinned separately by mel.npz)."""
    return (np.random.default_rng(11).standard_normal((1, 80, 6500)) * 0.5).astype(np.float32)


def batched_longform_features():
    """Three recordings of different lengths for the batched long-form fixtures (HF generate on the batch with an
    attention mask, run_eval.py:667-671): 65 s, 41.3 s and 18.2 s of independent deterministic draws, zero-padded to
    the longest -> (features [3, 80, 6500], attention mask [3, 6500])."""
    lens = [6500, 4130, 1820]
    feats = np.zeros((3, 80, 6500), dtype=np.float32)
    mask = np.zeros((3, 6500), dtype=np.int64)
    for i, n in enumerate(lens):
        feats[i, :, :n] = (np.random.default_rng(100 + i).standard_normal((80, n)) * 0.5).astype(np.float32)
        mask[i, :n] = 1
    return feats, mask


# ------------------------------------------------------------------------------------------ large-v2 decode fixture
LV2_SEED = 61


def lv2_features():
    """Four 30 s synthetic clips (the bench's sine + noise recipe, different seeds and tone lengths) and a 45 s
    long-form input (the first 4 500 frames of longform_features' deterministic draw)."""
    short = logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(3, 14.0),
                                  logmel.synthetic_clip(5, 22.0), logmel.synthetic_clip(8, 30.0)])
    return short, longform_features()[:, :, :4500]


# Decode-parity recipe at real widths, round 6 (moderate dynamic range, input-sensitive, not
# chaotic).  make_weights' default scales give a decoder whose argmax does not depend on the audio at d = 1280.  Round 5
# made it audio-dependent with a near-hard cross-attention (q, k x 7: scores of std ~25 over 1500 frames) and large
# value paths (v, out x 14): a residual stream of ~2.4e3, logits of ~85, and a decoder so sensitive to rounding that
# HF's own fp16 and bf16 runs left its fp32 run within a few steps.  This recipe instead keeps the cross-attention soft
# (q, k x 2.5: scores of std ~3) and removes what made a soft attention input-INdependent: the mean encoder row.
# Measured per decoder layer on HF fp32 with the round-5 style weights, the cross-attention output was 149 (norm) of a
# constant -- v of the mean encoder row, the same for every step and clip -- against 22 of a varying part.  The
# value bias of every cross-attention layer is set to -W_v . e_bar (e_bar = the mean HF fp32 encoder output row over
# the fixture's four 30 s clips, stored in the fixture as `v_bias`), so the attended frames' DIFFERENCE from the mean
# carries into the residual stream.  Measured on HF at these dims (fp32 greedy, 48 steps x 4 clips): 36-41 distinct
# tokens per row, a different row per clip, decoder residual stream max 25, logits max 22 (std 4.3), top-2 margin
# median 0.78; HF fp16 teacher-forced along HF fp32's tokens: logit rms distance 0.016, argmax agreement 99.5 %; HF bf16
# autocast: 0.106, 93.8 %.
LV2_DECODE_SCALES = {
    "decoder.embed_tokens.weight": 0.12 / 0.6,   # std 0.12 (logits of std ~4)
    "encoder_attn.q_proj.weight": 2.5,
    "encoder_attn.k_proj.weight": 2.5,
    "encoder_attn.v_proj.weight": 2.5,
    "encoder_attn.out_proj.weight": 2.5,
    "decoder.embed_positions.weight": 25.0,      # std 0.5: each step queries different frames
}


def lv2_decode_weights(cfg: dict, seed: int, v_bias=None) -> dict:
    """make_weights(cfg, seed, per_tensor=True, embed_std=0.6) with LV2_DECODE_SCALES applied to the decoder keys and,
    given v_bias [decoder_layers, d] (the fixture's `v_bias`), each cross-attention value bias replaced by its row."""
    w = make_weights(cfg, seed, per_tensor=True, embed_std=0.6)
    for k in w:
        if not k.startswith("model.decoder"):
            continue
        for pat, s in LV2_DECODE_SCALES.items():
            if k.endswith(pat):
                w[k] = (w[k] * np.float32(s)).astype(np.float32)
    if v_bias is not None:
        for i in range(cfg["decoder_layers"]):
            w[f"model.decoder.layers.{i}.encoder_attn.v_proj.bias"] = np.ascontiguousarray(v_bias[i], dtype=np.float32)
    return w


# ------------------------------------------------------------------------------ BASELINE-config parity fixtures
EMBED_STD = 0.05
CFG_CASES = {
    # c1: tiny <- tiny, B 2, launcher flags (freeze_encoder -> shared encoder, frozen decoder positions)
    "c1": dict(student="tiny", teacher="tiny", s_seed=31, t_seed=32, B=2, freeze_encoder=True,
               freeze_embed_positions=True, label_seed=41, secs=[30.0, 17.0]),
    # c2: small <- large-v2 (d 768 vs 1280: no sharing, full teacher forward), every student weight
    # trainable incl. the conv stem and encoder (240.6 M trainable)
    "c2": dict(student="small", teacher="large-v2", s_seed=33, t_seed=34, B=1, freeze_encoder=False,
               freeze_embed_positions=False, label_seed=42, secs=[30.0]),
    # c3: distil-32-2 made by create_student_model from the large-v2 teacher (decoder layers 0 and 31),
    # frozen shared encoder, a <|startofprev|> prompt (A7 teacher-input quirk at full size)
    "c3": dict(student=None, teacher="large-v2", s_seed=None, t_seed=34, B=1, freeze_encoder=True,
               freeze_embed_positions=True, label_seed=43, secs=[30.0], prompt=True),
    # c3 at B = 10: encoder rows 15 000 and decoder rows 4 470, the encoder projections on the persistent kernel of
    # the B = 64 step
    "c3b10": dict(student=None, teacher="large-v2", s_seed=None, t_seed=34, B=10, freeze_encoder=True,
                  freeze_embed_positions=True, label_seed=45, secs=[30.0, 27.5, 12.0, 30.0, 8.0, 19.0, 30.0, 24.0,
                                                                    30.0, 15.5], prompt=True),
}


def cfg_case_weights(case):
    """(student cfg, student weights, teacher cfg, teacher weights) of a BASELINE-config case."""
    from .student_ref import init_student_from_teacher
    c = CFG_CASES[case]
    tcfg = CONFIGS[c["teacher"]]
    wt = make_weights(tcfg, c["t_seed"], per_tensor=True, embed_std=EMBED_STD)
    if c["student"] is None:
        scfg, ws, _, _ = init_student_from_teacher(tcfg, wt, decoder_layers=2)
    else:
        scfg = CONFIGS[c["student"]]
        ws = make_weights(scfg, c["s_seed"], per_tensor=True, embed_std=EMBED_STD)
    return scfg, ws, tcfg, wt


def cfg_case_batch(case):
    c = CFG_CASES[case]
    feats = logmel.log_mel_batch([logmel.synthetic_clip(i, c["secs"][i]) for i in range(c["B"])])
    lists = L.synthetic_label_lists(c["B"], seed=c["label_seed"], prompt_fraction=0.0)
    if c.get("prompt"):
        lists[0] = [SPECIAL["startofprev"]] + list(range(300, 340)) + lists[0][:300]
    dec, lab = L.collate(lists)
    return feats, dec, lab
