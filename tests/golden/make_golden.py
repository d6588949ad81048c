"""Generate the golden parity fixtures from the REAL reference arithmetic.

Run in the build container (NOT on the GPU box; it needs /root/reference and the
HF Transformers oracle):   python tests/golden/make_golden.py

What produces each vector:
  * HF Transformers 5.15 `WhisperFeatureExtractor` (the reference's log-mel,
    `training/run_distillation.py:1217`)                                -> mel.npz
  * HF `WhisperForConditionalGeneration` fp32 on the micro config with the
    documented PRNG weights (oracle/weights.py); the reference's train_step
    arithmetic (`run_distillation.py:1507-1551`) applied to the HF outputs, the
    HF-model autograd backward and torch clip_grad_norm_ + AdamW
    (`:1425-1455,1666-1668`)                                            -> micro_step.npz
  * the reference's own `init_student_model_from_teacher`
    (`training/create_student_model.py:99-226`, imported from /root/reference)
    and `mix_language_embeddings` (`utils/model_utils.py:4-14`)         -> student.npz
  * HF `generate(num_beams=1)` greedy with forced prompt                 -> greedy.npz
  * the same forward / greedy / timestamp / long-form runs with torch_dtype=float16 -> fp16.npz
  * HF generate at the real large-v2 dims (fp32 and float16): greedy, timestamps, long-form gates
                                                                         -> lv2_decode.npz

Only small slices / checksums are stored (fixtures are data, no reference source).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import labels as L  # noqa: E402
from oracle import logmel  # noqa: E402
from oracle.weights import CONFIGS, SPECIAL, make_weights  # noqa: E402
# the fixtures' inputs and settings as plain data, shared with the GPU tests (which import neither this file nor HF)
from oracle.fixture_inputs import (CFG_CASES, EMBED_STD, LV2_GREEDY_GENERATION, LV2_SEED, ROWS, SUPPRESS,  # noqa: E402,F401
                                   TS_GENERATION, VSTRIDE, batched_longform_features, cfg_case_batch,
                                   cfg_case_weights, longform_features, lv2_decode_weights, lv2_features)

REF = "/root/reference"


def hf_model(cfg, w, dtype=torch.float32):
    from transformers import WhisperConfig, WhisperForConditionalGeneration
    m = WhisperForConditionalGeneration(WhisperConfig(**cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
    assert m.proj_out.weight.data_ptr() == m.model.decoder.embed_tokens.weight.data_ptr()
    return m.to(dtype)


def micro_batch():
    feats = logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(1, 17.0)])
    lists = L.synthetic_label_lists(2, seed=0)
    # force a <|startofprev|> prompt on clip 1 (exercise the A7 teacher-input quirk)
    lists[1] = [SPECIAL["startofprev"], 11, 12, 13] + lists[1][:200]
    dec, lab = L.collate(lists)
    return feats, dec, lab, lists


def gen_mel(out):
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor()
    clips = [logmel.synthetic_clip(0), logmel.synthetic_clip(3, 12.0), logmel.synthetic_clip(5, 45.0)]
    clips.append(np.zeros(16000, dtype=np.float32))   # silent clip: floor path
    mel = fe(clips, sampling_rate=16000, return_tensors="np").input_features.astype(np.float32)
    out["mel_sub"] = mel[:, :, ::10]
    out["mel_rowsum"] = mel.sum(-1)
    out["mel_max"] = mel.reshape(len(clips), -1).max(-1)
    out["mel_filters"] = fe.mel_filters.astype(np.float32)


def longform_clips():
    """Two long-form clips of different lengths (47.3 s, 65 s: not a multiple of the hop)."""
    return [logmel.synthetic_clip(6, 47.3), logmel.synthetic_clip(7, 65.0)]


def gen_mel_long(out):
    """HF long-form feature extraction as run_eval.py:572-581 calls it (truncation=False,
    padding="longest", return_attention_mask=True)."""
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor()
    r = fe(longform_clips(), sampling_rate=16000, return_tensors="np", truncation=False, padding="longest",
           return_attention_mask=True)
    mel = r.input_features.astype(np.float32)
    out["mel_sub"] = mel[:, :, ::10]
    out["mel_rowsum"] = mel.sum(-1)
    out["mel_max"] = mel.reshape(mel.shape[0], -1).max(-1)
    out["shape"] = np.array(mel.shape)
    out["attention_mask"] = np.asarray(r.attention_mask).astype(np.int8)


def gen_micro(out):
    from transformers.modeling_outputs import BaseModelOutput
    cfg = CONFIGS["micro"]
    ws, wt = make_weights(cfg, 1), make_weights(cfg, 2)
    S, Tm = hf_model(cfg, ws), hf_model(cfg, wt)
    feats, dec, lab, _ = micro_batch()
    feats_t, dec_t, lab_t = torch.from_numpy(feats), torch.from_numpy(dec), torch.from_numpy(lab)
    out["feats"], out["dec"], out["lab"] = feats, dec, lab
    S.eval(); Tm.eval()
    # freeze student encoder (c3 recipe: share_hidden_states, run_distillation.py:1043-1075)
    for p in S.model.encoder.parameters():
        p.requires_grad_(False)
    S.model.decoder.embed_positions.weight.requires_grad_(False)
    so = S(input_features=feats_t, decoder_input_ids=dec_t, labels=lab_t)
    with torch.no_grad():
        to_share = Tm(encoder_outputs=BaseModelOutput(so.encoder_last_hidden_state.detach()), labels=lab_t)
        to_full = Tm(input_features=feats_t, decoder_input_ids=dec_t, labels=lab_t)
    T = 2.0

    def kl_of(t_logits):
        p = torch.softmax(t_logits / T, -1)
        lq = torch.log_softmax(so.logits / T, -1)
        div = torch.nn.functional.kl_div(lq, p, reduction="none") * (lab_t >= 0).unsqueeze(-1)
        return div.sum() / (lab_t >= 0).sum() * T ** 2

    kl_share, kl_full = kl_of(to_share.logits), kl_of(to_full.logits)
    loss = 0.8 * so.loss + 1.0 * kl_share
    out["ce"], out["kl_share"], out["kl_full"], out["loss"] = [np.float64(x.item()) for x in
                                                               (so.loss, kl_share, kl_full, loss)]
    out["enc_sub"] = so.encoder_last_hidden_state.detach().numpy()[:, ::50, :]
    lg = so.logits.detach()
    out["s_lse"] = torch.logsumexp(lg, -1).numpy()
    out["s_argmax"] = lg.argmax(-1).numpy()
    out["s_rows"] = lg[:, ROWS, ::VSTRIDE].numpy()
    out["t_share_lse"] = torch.logsumexp(to_share.logits, -1).numpy()
    out["t_share_rows"] = to_share.logits[:, ROWS, ::VSTRIDE].numpy()
    out["t_full_lse"] = torch.logsumexp(to_full.logits, -1).numpy()
    loss.backward()
    names = [n for n, p in S.named_parameters() if p.requires_grad]
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array([S.get_parameter(n).grad.norm().item() for n in names])
    g = S.model.decoder.layers[1].fc2.weight.grad
    out["grad_dec1_fc2_sub"] = g[::7, ::11].clone().numpy()
    out["grad_embed_rows"] = S.model.decoder.embed_tokens.weight.grad[[50258, 50260, 50363, 11, 12]].clone().numpy()
    # clip + AdamW (lr 1e-4) one update, as the reference loop does on the sync step
    tp = [S.get_parameter(n) for n in names]
    gn = torch.nn.utils.clip_grad_norm_(tp, 1.0)
    opt = torch.optim.AdamW(tp, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
    opt.step()
    out["grad_total_norm"] = np.float64(gn.item())
    out["upd_dec0_q_sub"] = S.model.decoder.layers[0].self_attn.q_proj.weight.detach()[::5, ::5].numpy()
    out["upd_embed_row"] = S.model.decoder.embed_tokens.weight.detach()[[50260, 100]].numpy()
    # the same student forward under bf16 autocast (the reference's mixed_precision="bf16" path, see
    # gen_cfg): the size of the reference's own bf16 noise on this model
    S2 = hf_model(cfg, ws).eval()
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        so2 = S2(input_features=feats_t, decoder_input_ids=dec_t, labels=lab_t)
    out["amp_ce"] = np.float64(so2.loss.float().item())
    out["amp_enc_sub"] = so2.encoder_last_hidden_state.float().numpy()[:, ::50, :]
    out["amp_s_lse"] = torch.logsumexp(so2.logits.float(), -1).numpy()


def gen_student(out):
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "training"))
    import create_student_model as csm      # reference module (imports utils.model_utils)
    from transformers import WhisperFeatureExtractor

    class _Proc:  # tokenizer files are absent offline: stub processor
        def __init__(self):
            self.feature_extractor = WhisperFeatureExtractor()
            self.tokenizer = types.SimpleNamespace(
                convert_tokens_to_ids=lambda t: {"<|en|>": SPECIAL["en"], "<|zh|>": SPECIAL["zh"]}[t])

        @classmethod
        def from_pretrained(cls, *a, **k):
            return cls()

        def save_pretrained(self, *a, **k):
            pass

        def __call__(self, audio, sampling_rate=16000, return_tensors="pt"):
            return self.feature_extractor(audio, sampling_rate=sampling_rate, return_tensors=return_tensors)

    csm.WhisperProcessor = _Proc
    from transformers import GenerationConfig
    cfg = dict(CONFIGS["micro"], encoder_layers=4, decoder_layers=5)
    w = make_weights(cfg, 7)
    tmp = tempfile.mkdtemp()
    tdir, sdir = os.path.join(tmp, "teacher"), os.path.join(tmp, "student")
    hf_model(cfg, w).save_pretrained(tdir)
    GenerationConfig(decoder_start_token_id=SPECIAL["sot"]).save_pretrained(tdir)
    cases = {"e2_d2": dict(encoder_layers=2, decoder_layers=2),
             "d3": dict(decoder_layers=3),
             "e3_dnums": dict(encoder_layers=3, decoder_layers=2, decoder_layers_numbers=[1, 4]),
             "mix": dict(encoder_layers=2, decoder_layers=2, mix_lang_emb=True)}
    from safetensors.numpy import load_file
    meta = {}
    for name, kw in cases.items():
        d = sdir + "_" + name
        csm.init_student_model_from_teacher(tdir, save_dir=d, **kw)
        sd = load_file(os.path.join(d, "model.safetensors"))
        scfg = json.load(open(os.path.join(d, "config.json")))
        meta[name] = dict(encoder_layers=scfg["encoder_layers"], decoder_layers=scfg["decoder_layers"],
                          keys=sorted(sd))
        for k in sorted(sd):
            out[f"{name}|{k}"] = np.float64(np.asarray(sd[k], dtype=np.float64).sum())
    out["student_meta"] = np.array(json.dumps(meta))
    # mix_language_embeddings on a bf16 teacher (the reference's teacher dtype, :1019-1020)
    from utils.model_utils import mix_language_embeddings
    m = hf_model(cfg, w).to(torch.bfloat16)
    tok = types.SimpleNamespace(convert_tokens_to_ids=lambda t: {"<|en|>": SPECIAL["en"], "<|zh|>": SPECIAL["zh"]}[t])
    mix_language_embeddings(m, tok, languages=["zh", "en"])
    out["mix_bf16_row_u16"] = m.model.decoder.embed_tokens.weight[SPECIAL["zh"]].view(torch.int16).numpy()
    m32 = hf_model(cfg, w)
    mix_language_embeddings(m32, tok, languages=["en", "zh"], weights=[0.5, 0.5])
    out["mix_f32_row"] = m32.model.decoder.embed_tokens.weight[SPECIAL["zh"]].detach().numpy()


def gen_greedy(out):
    from transformers import GenerationConfig
    cfg = CONFIGS["micro"]
    m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2)).eval()   # stronger layers: non-trivial decode
    feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0),
                                                   logmel.synthetic_clip(4, 25.0)]))
    prompt = [SPECIAL["sot"], SPECIAL["zh"], SPECIAL["transcribe"], SPECIAL["notimestamps"]]
    gc = GenerationConfig(decoder_start_token_id=SPECIAL["sot"], eos_token_id=SPECIAL["eot"],
                          pad_token_id=SPECIAL["pad"], suppress_tokens=SUPPRESS,
                          begin_suppress_tokens=[220, SPECIAL["eot"]], max_length=64, num_beams=1,
                          do_sample=False, no_timestamps_token_id=SPECIAL["notimestamps"])
    m.generation_config = gc
    with torch.no_grad():
        ids = m.generate(feats, decoder_input_ids=torch.tensor([prompt] * 3), max_length=64,
                         num_beams=1, do_sample=False)
    out["greedy_ids"] = ids.numpy()        # HF returns the generated tokens only (prompt stripped)
    out["greedy_prompt"] = np.array(prompt)
    out["suppress"] = np.array(SUPPRESS)


def gen_beam(out):
    """HF `generate(num_beams=k)` (short-form, forced prompt, no timestamps) on the greedy fixture's model and clips:
    the beam search of `training/run_eval.py:144-147` / `run_distillation.py:1476-1484` (GenerationMixin._beam_search:
    log-softmax, the suppress processors on log-probs, 2k candidates, length penalty 1.0, early_stopping False).
    Two weight sets: the greedy fixture's (every beam runs to max_length) and the same with the <|endoftext|> row of the
    tied embedding scaled by 6 (beams finish at different steps: the finished-hypotheses path)."""
    from transformers import GenerationConfig
    cfg = CONFIGS["micro"]
    feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0),
                                                   logmel.synthetic_clip(4, 25.0)]))
    prompt = [SPECIAL["sot"], SPECIAL["zh"], SPECIAL["transcribe"], SPECIAL["notimestamps"]]
    for tag, eos_scale in (("", 1.0), ("_eos6", 6.0)):
        w = make_weights(cfg, 1, lin_std=0.2)
        w["model.decoder.embed_tokens.weight"] = w["model.decoder.embed_tokens.weight"].copy()
        w["model.decoder.embed_tokens.weight"][SPECIAL["eot"]] *= eos_scale
        m = hf_model(cfg, w).eval()
        for nb in (2, 4):
            gc = GenerationConfig(decoder_start_token_id=SPECIAL["sot"], eos_token_id=SPECIAL["eot"],
                                  pad_token_id=SPECIAL["pad"], suppress_tokens=SUPPRESS,
                                  begin_suppress_tokens=[220, SPECIAL["eot"]], max_length=64, num_beams=nb,
                                  do_sample=False, no_timestamps_token_id=SPECIAL["notimestamps"])
            m.generation_config = gc
            with torch.no_grad():
                ids = m.generate(feats, decoder_input_ids=torch.tensor([prompt] * 3), max_length=64, num_beams=nb,
                                 do_sample=False)
            out[f"beam{nb}{tag}_ids"] = ids.numpy()      # generated tokens only, finished rows padded with eos
    out["beam_prompt"] = np.array(prompt)
    out["beam_eos_scale"] = np.float32(6.0)


def gen_beam_ts(out):
    """HF `generate(num_beams=k, return_timestamps=True)` on the timestamp fixtures' micro model (lin_std 0.2): the
    seek loop with a beam search per window (generate_with_fallback: the temperature-0 attempt keeps num_beams), the
    timestamp processor on the log-probs, HF's beam _postprocess_outputs (the chosen beam's per-step scores through
    beam_indices) for the gates.
      bts{k}_short_ids : 2 clips <= 30 s, language zh, max_new_tokens 48
      bts{k}_long_ids, bts{k}_long_avg_logprobs, bts{k}_long_ns_probs : the 65 s input, temperature (0.0,), thresholds
                         that never fire (logprob -1e9, no-speech 1.0), per-window gates recorded in _need_fallback"""
    cfg = CONFIGS["micro"]
    m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2)).eval()
    feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0)]))
    lf = torch.from_numpy(longform_features())
    am = torch.ones(1, lf.shape[-1], dtype=torch.long)
    for k in (2, 4):
        m.generation_config = ts_generation_config()
        with torch.no_grad():
            out[f"bts{k}_short_ids"] = m.generate(feats, return_timestamps=True, language="zh", task="transcribe",
                                                  max_new_tokens=48, num_beams=k).numpy()
        rec = {"avg": [], "ns": []}
        orig_need = type(m)._need_fallback

        def spy(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size,
                temperature):
            rec["avg"].append(float(self._retrieve_avg_logprobs(seek_outputs[index]["scores"], seek_sequence,
                                                                temperature)))
            from transformers.generation.logits_process import WhisperNoSpeechDetection
            for p_ in logits_processor or []:
                if isinstance(p_, WhisperNoSpeechDetection):
                    rec["ns"].append(float(p_.no_speech_prob[index]))
            return orig_need(self, seek_sequence, seek_outputs, index, logits_processor, generation_config,
                             vocab_size, temperature)
        m.generation_config = ts_generation_config()
        type(m)._need_fallback = spy
        try:
            with torch.no_grad():
                out[f"bts{k}_long_ids"] = m.generate(lf, attention_mask=am, return_timestamps=True, language="zh",
                                                     task="transcribe", num_beams=k, temperature=(0.0,),
                                                     logprob_threshold=-1e9, no_speech_threshold=1.0).numpy()
        finally:
            type(m)._need_fallback = orig_need
        out[f"bts{k}_long_avg_logprobs"] = np.array(rec["avg"], dtype=np.float64)
        out[f"bts{k}_long_ns_probs"] = np.array(rec["ns"], dtype=np.float64)
        print("beam_ts", k, "done", flush=True)


def ts_generation_config():
    from transformers import GenerationConfig
    return GenerationConfig(**TS_GENERATION)


def gen_greedy_ts(out):
    """HF generate(return_timestamps=True): short-form window and a 65 s long-form input."""
    cfg = CONFIGS["micro"]
    m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2)).eval()
    m.generation_config = ts_generation_config()
    feats = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0)]))
    with torch.no_grad():
        ids = m.generate(feats, return_timestamps=True, language="zh", task="transcribe", max_new_tokens=48)
    out["ts_short_ids"] = ids.numpy()
    lf = torch.from_numpy(longform_features())
    with torch.no_grad():
        ids = m.generate(lf, attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True,
                         language="zh", task="transcribe")
    out["ts_long_ids"] = ids.numpy()


def gen_fallback(out):
    """HF long-form generate with previous-text conditioning (temperature 0) and with the fallback
    thresholds at a single temperature (deterministic: no sampled retry), on the 65 s features:
      fb_cond_ids       condition_on_prev_tokens=True
      fb_none_ids       logprob_threshold=-1e9, no_speech_threshold=1.0   (no window fails / is skipped)
      fb_skipall_ids    logprob_threshold=+1e9, no_speech_threshold=0.0   (every window skipped)
      fb_ns_probs / fb_avg_logprobs: per-window no-speech probability and avg log-prob recorded from
                        HF's WhisperNoSpeechDetection / _retrieve_avg_logprobs during the cond run."""
    cfg = CONFIGS["micro"]
    m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2)).eval()
    m.generation_config = ts_generation_config()
    lf = torch.from_numpy(longform_features())
    am = torch.ones(1, lf.shape[-1], dtype=torch.long)
    kw = dict(attention_mask=am, return_timestamps=True, language="zh", task="transcribe")
    rec = {"avg": [], "ns": []}
    orig_need = type(m)._need_fallback

    def spy(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature):
        scores = seek_outputs[index]["scores"]
        rec["avg"].append(float(self._retrieve_avg_logprobs(scores, seek_sequence, temperature)))
        from transformers.generation.logits_process import WhisperNoSpeechDetection
        for p_ in logits_processor or []:
            if isinstance(p_, WhisperNoSpeechDetection):
                rec["ns"].append(float(p_.no_speech_prob[index]))
        return orig_need(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size,
                         temperature)
    with torch.no_grad():
        out["fb_cond_ids"] = m.generate(lf, condition_on_prev_tokens=True, temperature=0.0, **kw).numpy()
        out["fb_none_ids"] = m.generate(lf, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0,
                                        **kw).numpy()
        out["fb_skipall_ids"] = m.generate(lf, temperature=(0.0,), logprob_threshold=1e9, no_speech_threshold=0.0,
                                           **kw).numpy()
        type(m)._need_fallback = spy
        try:
            m.generate(lf, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0, **kw)
        finally:
            type(m)._need_fallback = orig_need
    out["fb_avg_logprobs"] = np.array(rec["avg"], dtype=np.float64)
    out["fb_ns_probs"] = np.array(rec["ns"], dtype=np.float64)


def gen_fp16(out):
    """HF Whisper with torch_dtype=float16 (no autocast) on CPU -- the arithmetic of the reference's fp16 decode
    call sites (run_eval.py:99 --dtype float16 default, :500-509 model.to(dtype), :589 input_features.to(dtype);
    run_pseudo_labelling.py:461-463 via run-pseudo-labelling.sh:30): fp16 weights, fp16 Linear / conv / SDPA
    outputs and residual stream, LayerNorm and GELU computed in fp32 with fp16 results, fp16 logits.
      f16_enc_sub / f16_s_rows / f16_s_lse: forward of the micro_step batch (micro weights, seed 1)
      f16_greedy_ids:   generate() greedy, the greedy.npz setup (lin_std 0.2 weights, 3 clips, max_length 64)
      f16_ts_short_ids / f16_ts_long_ids: the greedy_ts.npz setup (timestamps, 65 s long-form)
      f16_fb_cond_ids / f16_fb_avg_logprobs / f16_fb_ns_probs: the fallback.npz conditioned long-form run"""
    cfg = CONFIGS["micro"]
    # forward
    m = hf_model(cfg, make_weights(cfg, 1), torch.float16).eval()
    feats, dec, lab, _ = micro_batch()
    with torch.no_grad():
        o = m(input_features=torch.from_numpy(feats).half(), decoder_input_ids=torch.from_numpy(dec))
    out["f16_enc_sub"] = o.encoder_last_hidden_state.float().numpy()[:, ::50, :]
    lg = o.logits.float()
    out["f16_s_lse"] = torch.logsumexp(lg, -1).numpy()
    out["f16_s_argmax"] = lg.argmax(-1).numpy()
    out["f16_s_rows"] = lg[:, ROWS, ::VSTRIDE].numpy()
    # greedy
    from transformers import GenerationConfig
    m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2), torch.float16).eval()
    gfe = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0),
                                                 logmel.synthetic_clip(4, 25.0)])).half()
    prompt = [SPECIAL["sot"], SPECIAL["zh"], SPECIAL["transcribe"], SPECIAL["notimestamps"]]
    m.generation_config = GenerationConfig(decoder_start_token_id=SPECIAL["sot"], eos_token_id=SPECIAL["eot"],
                                           pad_token_id=SPECIAL["pad"], suppress_tokens=SUPPRESS,
                                           begin_suppress_tokens=[220, SPECIAL["eot"]], max_length=64, num_beams=1,
                                           do_sample=False, no_timestamps_token_id=SPECIAL["notimestamps"])
    with torch.no_grad():
        out["f16_greedy_ids"] = m.generate(gfe, decoder_input_ids=torch.tensor([prompt] * 3), max_length=64,
                                           num_beams=1, do_sample=False).numpy()
    # timestamps, long-form, conditioning + gates
    m.generation_config = ts_generation_config()
    tfe = torch.from_numpy(logmel.log_mel_batch([logmel.synthetic_clip(0), logmel.synthetic_clip(2, 9.0)])).half()
    lf = torch.from_numpy(longform_features()).half()
    am = torch.ones(1, lf.shape[-1], dtype=torch.long)
    kw = dict(return_timestamps=True, language="zh", task="transcribe")
    rec = {"avg": [], "ns": []}
    orig_need = type(m)._need_fallback

    def spy(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size, temperature):
        scores = seek_outputs[index]["scores"]
        rec["avg"].append(float(self._retrieve_avg_logprobs(scores, seek_sequence, temperature)))
        from transformers.generation.logits_process import WhisperNoSpeechDetection
        for p_ in logits_processor or []:
            if isinstance(p_, WhisperNoSpeechDetection):
                rec["ns"].append(float(p_.no_speech_prob[index]))
        return orig_need(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size,
                         temperature)
    with torch.no_grad():
        out["f16_ts_short_ids"] = m.generate(tfe, max_new_tokens=48, **kw).numpy()
        out["f16_ts_long_ids"] = m.generate(lf, attention_mask=am, **kw).numpy()
        out["f16_fb_cond_ids"] = m.generate(lf, attention_mask=am, condition_on_prev_tokens=True, temperature=0.0,
                                            **kw).numpy()
        type(m)._need_fallback = spy
        try:
            m.generate(lf, attention_mask=am, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0, **kw)
        finally:
            type(m)._need_fallback = orig_need
    out["f16_fb_avg_logprobs"] = np.array(rec["avg"], dtype=np.float64)
    out["f16_fb_ns_probs"] = np.array(rec["ns"], dtype=np.float64)


class _MarginSpy:
    """A logits processor appended after HF's own (generate merges a custom processor list after the built-in
    ones): records, per decode step and row, the gap between the two largest PROCESSED scores -- how close the
    greedy choice was to a tie."""

    def __init__(self):
        self.steps = []

    def __call__(self, input_ids, scores):
        top = scores.float().topk(2, dim=-1).values
        self.steps.append((top[:, 0] - top[:, 1]).numpy().astype(np.float32))
        return scores


def lv2_greedy_config():
    from transformers import GenerationConfig
    return GenerationConfig(**LV2_GREEDY_GENERATION)


def _lv2_tf_logits(m, feats, full_ids, amp):
    """HF teacher-forced forward: logits [B, T, V] (fp32) of decoder_input_ids = full_ids."""
    with torch.no_grad(), amp:
        return m(input_features=feats, decoder_input_ids=full_ids).logits.float()


def gen_lv2_decode(out):
    """HF generate at the REAL large-v2 dimensions (d 1280, 32 + 32 layers, 20 heads) -- the model of BASELINE c4 / c5
    -- with the round-6 decode-parity weights (oracle/fixture_inputs.lv2_decode_weights(large-v2, LV2_SEED, v_bias):
    a soft cross-attention whose value path carries each step's attended frames' difference from the mean encoder
    row; moderate range, audio-dependent, not chaotic -- see LV2_DECODE_SCALES), in three arithmetics:
      f32  fp32 model (mixed_precision "no")
      f16  torch_dtype=float16 model, no autocast (run_eval.py:99, run_pseudo_labelling.py:461-463)
      b16  fp32 model under torch.autocast("cpu", bfloat16) (run_distillation.py:1580-1584: generate_step runs the
           student under the bf16 Accelerator)
    Stored:
      v_bias                     : [32, 1280] cross-attention value biases, -W_v . e_bar, e_bar = the mean HF fp32
                                   encoder output row of the four 30 s clips (part of the weight recipe)
      {tag}_greedy_ids / _margin : free-running greedy, 4 clips, [SOT, zh, transcribe, notimestamps], 48 new tokens
                                   (run_pseudo_labelling.py:917-922 without timestamps); margin = per step and row,
                                   top-1 minus top-2 processed score (_MarginSpy)
      {tag}_ts_ids / _margin     : return_timestamps=True, language zh, 48 new tokens, one clip per call (rows padded
                                   with -1; margins [step, clip], nan-padded)
      tf_*                       : TEACHER-FORCED along HF fp32's greedy tokens (one forward over prompt + tokens, the
                                   logits at the S = 48 predicting positions): tf_len [B] steps up to and including a
                                   row's eos; tf_top_ids [B, S, 16] the 16 largest PROCESSED (suppress tokens masked,
                                   begin tokens at step 0) HF fp32 scores; tf_{tag}_vals [B, S, 16] each arithmetic's
                                   RAW logits at those ids; tf_{tag}_lse [B, S] logsumexp of the raw row;
                                   tf_{tag}_argmax / _margin [B, S] argmax and top-2 gap of the processed row;
                                   tf_oracle{16,b16}_vals: the same values from the CPU oracle (oracle/whisper_ref.Ref
                                   with the engine's 16-bit rounding points) -- the a-priori distance of a correct
                                   rounding model from HF, recorded beside the tests' bars
      f32_long_*                 : 45 s long-form (fp32), temperature (0.0,), thresholds that never fire, per-window
                                   gates and margins (run_eval.py:659-665)"""
    import contextlib
    from transformers.generation.logits_process import LogitsProcessorList
    from oracle.whisper_ref import Ref
    cfg = CONFIGS["large-v2"]
    d, Ldec = cfg["d_model"], cfg["decoder_layers"]
    short, lf = lv2_features()
    prompt = [SPECIAL["sot"], SPECIAL["zh"], SPECIAL["transcribe"], SPECIAL["notimestamps"]]
    P, B, S, K = len(prompt), short.shape[0], 48, 16
    w = lv2_decode_weights(cfg, LV2_SEED)
    m = hf_model(cfg, w).eval()
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(short)).last_hidden_state
    ebar = enc.reshape(-1, d).double().mean(0)
    v_bias = np.stack([-(torch.from_numpy(w[f"model.decoder.layers.{i}.encoder_attn.v_proj.weight"]).double() @ ebar)
                       .float().numpy() for i in range(Ldec)])
    out["v_bias"] = v_bias
    w = lv2_decode_weights(cfg, LV2_SEED, v_bias)
    del m, enc
    sup = torch.tensor(LV2_GREEDY_GENERATION["suppress_tokens"])

    def processed(lg):
        lg = lg.clone()
        lg[..., sup] = -float("inf")
        lg[:, 0, [220, SPECIAL["eot"]]] = -float("inf")
        return lg
    full = None
    for dt, tag in ((torch.float32, "f32"), (torch.float16, "f16"), (torch.float32, "b16")):
        m = hf_model(cfg, w, dt).eval()
        amp = torch.autocast("cpu", dtype=torch.bfloat16) if tag == "b16" else contextlib.nullcontext()
        feats = torch.from_numpy(short).to(dt)
        m.generation_config = lv2_greedy_config()
        spy = _MarginSpy()
        with torch.no_grad(), amp:
            ids = m.generate(feats, decoder_input_ids=torch.tensor([prompt] * B), max_new_tokens=S,
                             logits_processor=LogitsProcessorList([spy])).numpy()
        out[f"{tag}_greedy_ids"] = ids
        out[f"{tag}_greedy_margin"] = np.stack(spy.steps)
        if tag == "f32":
            gen = np.pad(ids, ((0, 0), (0, S - ids.shape[1])), constant_values=SPECIAL["eot"])   # generated ids only
            out["tf_len"] = np.array([list(r).index(SPECIAL["eot"]) + 1 if SPECIAL["eot"] in r else S for r in gen])
            full = torch.from_numpy(np.concatenate([np.array([prompt] * B), gen[:, :S - 1]], 1))
        lg = _lv2_tf_logits(m, feats, full, amp)[:, P - 1:P - 1 + S]            # [B, S, V]
        pl = processed(lg)
        if tag == "f32":
            top = pl.topk(K, dim=-1).indices
            out["tf_top_ids"] = top.numpy().astype(np.int32)
        out[f"tf_{tag}_vals"] = torch.gather(lg, -1, top).numpy()
        out[f"tf_{tag}_lse"] = torch.logsumexp(lg, -1).numpy()
        t2 = pl.topk(2, dim=-1)
        out[f"tf_{tag}_argmax"] = t2.indices[..., 0].numpy().astype(np.int32)
        out[f"tf_{tag}_margin"] = (t2.values[..., 0] - t2.values[..., 1]).numpy()
        del lg, pl
        m.generation_config = ts_generation_config()
        # one clip per call: HF's timestamp path drops finished rows from its batch (_maybe_reduce_batch), so a
        # batched call's per-step margins cannot be mapped back to clips; rows are padded with -1 / nan
        ids_l, mar_l = [], []
        for b in range(B):
            spy = _MarginSpy()
            with torch.no_grad(), amp:
                ids_l.append(m.generate(feats[b:b + 1], return_timestamps=True, language="zh", task="transcribe",
                                        max_new_tokens=S, logits_processor=LogitsProcessorList([spy])).numpy()[0])
            mar_l.append(np.concatenate([s_.reshape(-1) for s_ in spy.steps]))
        L_ = max(len(x) for x in ids_l)
        out[f"{tag}_ts_ids"] = np.stack([np.pad(x, (0, L_ - len(x)), constant_values=-1) for x in ids_l])
        S_ = max(len(x) for x in mar_l)
        out[f"{tag}_ts_margin"] = np.stack([np.pad(x, (0, S_ - len(x)), constant_values=np.nan) for x in mar_l]).T
        print(tag, "greedy + teacher-forced + timestamps done", flush=True)
        if tag == "f32":
            lt = torch.from_numpy(lf).to(dt)
            kw = dict(attention_mask=torch.ones(1, lt.shape[-1], dtype=torch.long), return_timestamps=True,
                      language="zh", task="transcribe")
            rec = {"avg": [], "ns": [], "steps": [], "raw": []}
            orig_need = type(m)._need_fallback

            def need_spy(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size,
                         temperature):
                rec["steps"].append(len(seek_outputs[index]["scores"]))
                rec["raw"].append([int(t) for t in seek_sequence.tolist()])
                rec["avg"].append(float(self._retrieve_avg_logprobs(seek_outputs[index]["scores"], seek_sequence,
                                                                    temperature)))
                from transformers.generation.logits_process import WhisperNoSpeechDetection
                for p_ in logits_processor or []:
                    if isinstance(p_, WhisperNoSpeechDetection):
                        rec["ns"].append(float(p_.no_speech_prob[index]))
                return orig_need(self, seek_sequence, seek_outputs, index, logits_processor, generation_config,
                                 vocab_size, temperature)
            type(m)._need_fallback = need_spy
            spy = _MarginSpy()
            try:
                with torch.no_grad():
                    out[f"{tag}_long_ids"] = m.generate(lt, temperature=(0.0,), logprob_threshold=-1e9,
                                                        no_speech_threshold=1.0,
                                                        logits_processor=LogitsProcessorList([spy]), **kw).numpy()
            finally:
                type(m)._need_fallback = orig_need
            out[f"{tag}_long_avg_logprobs"] = np.array(rec["avg"], dtype=np.float64)
            out[f"{tag}_long_ns_probs"] = np.array(rec["ns"], dtype=np.float64)
            out[f"{tag}_long_window_steps"] = np.array(rec["steps"], dtype=np.int64)
            # each window's tokens as HF's gate saw them (seek_sequence), -1-padded [window, token]
            Lw = max(len(r_) for r_ in rec["raw"])
            out[f"{tag}_long_window_ids"] = np.array([r_ + [-1] * (Lw - len(r_)) for r_ in rec["raw"]], dtype=np.int64)
            # one row per decode step over all windows, in order (batch of one)
            out[f"{tag}_long_margin"] = np.concatenate([s_.reshape(-1) for s_ in spy.steps])
            print(tag, "long-form done", flush=True)
        del m
    # the CPU oracle with the engine's rounding points, teacher-forced along the same tokens
    wt = {k: torch.from_numpy(v) for k, v in w.items()}
    for name, kw in (("oracle16", dict(amp=True, stream_bf16=True, half=torch.float16)),
                     ("oracleb16", dict(amp=True, stream_bf16=False, half=torch.bfloat16))):
        ref = Ref(cfg, wt, **kw)
        with torch.no_grad():
            lg = ref.forward(feats=torch.from_numpy(short), decoder_input_ids=full)["logits"][:, P - 1:P - 1 + S]
        out[f"tf_{name}_vals"] = torch.gather(lg, -1, top).numpy()
        print(name, "done", flush=True)
    out["prompt"] = np.array(prompt)
    out["seed"] = np.int64(LV2_SEED)


def gen_batched_longform(out):
    """HF's BATCHED sequential long-form generate (generation_whisper.py:785-898 + generate_with_fallback :970-1117):
    ONE generate call on 3 recordings of different lengths (oracle/fixture_inputs.batched_longform_features: 65 s,
    41.3 s, 18.2 s, attention mask), the call of run_eval.py:667-681 (return_timestamps, language zh, temperature
    (0.0,), thresholds that never fire so every window's gates are recorded but none falls back), in fp32 at
      micro  the timestamp fixture's micro model (make_weights(micro, 1, lin_std=0.2), greedy_ts.npz)
      lv2    the large-v2 decode-parity model (lv2_decode_weights with lv2_decode.npz's v_bias)
    Stored per {dims}: bl_{dims}_ids (the call's output, pad-padded); per decoded window in HF's order (seek iteration,
    then batch row): bl_{dims}_win_b (recording), _win_seek (frame), _win_ids (the tokens HF's gate saw, -1-padded),
    _win_avg / _win_ns (average log-prob, no-speech probability), _win_margin (per step top-1 minus top-2 processed
    score, nan-padded); the batch of each iteration is recorded by spying on _maybe_reduce_batch."""
    from transformers.generation.logits_process import LogitsProcessorList, WhisperNoSpeechDetection
    feats, mask = batched_longform_features()
    prev = os.path.join(HERE, "batched_longform.npz")         # BL_DIMS=lv2 (say) keeps the other dims' arrays
    if os.path.exists(prev):
        z = np.load(prev)
        out.update({k_: z[k_] for k_ in z.files})
    lv2 = np.load(os.path.join(HERE, "lv2_decode.npz"))
    for dims in os.environ.get("BL_DIMS", "micro,lv2").split(","):
        if dims == "micro":
            cfg = CONFIGS["micro"]
            m = hf_model(cfg, make_weights(cfg, 1, lin_std=0.2)).eval()
        else:
            cfg = CONFIGS["large-v2"]
            m = hf_model(cfg, lv2_decode_weights(cfg, int(lv2["seed"]), lv2["v_bias"])).eval()
        m.generation_config = ts_generation_config()
        cls = type(m)
        orig_need, orig_red = cls._need_fallback, cls._maybe_reduce_batch
        rec = {"b": [], "seek": [], "ids": [], "avg": [], "ns": [], "margin": []}
        it = {"map": None, "seek": None, "start": 0}
        spy = _MarginSpy()

        def red_spy(input_features, seek, max_frames, cur_bsz, batch_idx_map):
            r = orig_red(input_features, seek, max_frames, cur_bsz, batch_idx_map)
            it["map"], it["seek"], it["start"] = list(r[2]), seek.clone(), len(spy.steps)
            return r

        def need_spy(self, seek_sequence, seek_outputs, index, logits_processor, generation_config, vocab_size,
                     temperature):
            b = it["map"][index]
            rec["b"].append(b)
            rec["seek"].append(int(it["seek"][b]))
            rec["ids"].append([int(t) for t in seek_sequence.tolist()])
            rec["avg"].append(float(self._retrieve_avg_logprobs(seek_outputs[index]["scores"], seek_sequence,
                                                                temperature)))
            for p_ in logits_processor or []:
                if isinstance(p_, WhisperNoSpeechDetection):
                    rec["ns"].append(float(p_.no_speech_prob[index]))
            steps = spy.steps[it["start"]:]
            rec["margin"].append(np.array([s_[index] for s_ in steps[:len(seek_outputs[index]["scores"])]],
                                          dtype=np.float32))
            return orig_need(self, seek_sequence, seek_outputs, index, logits_processor, generation_config,
                             vocab_size, temperature)
        cls._need_fallback, cls._maybe_reduce_batch = need_spy, staticmethod(red_spy)
        try:
            with torch.no_grad():
                ids = m.generate(torch.from_numpy(feats), attention_mask=torch.from_numpy(mask), return_timestamps=True,
                                 language="zh", task="transcribe", temperature=(0.0,), logprob_threshold=-1e9,
                                 no_speech_threshold=1.0, logits_processor=LogitsProcessorList([spy])).numpy()
        finally:
            cls._need_fallback, cls._maybe_reduce_batch = orig_need, staticmethod(orig_red)
        k = f"bl_{dims}"
        out[f"{k}_ids"] = ids
        out[f"{k}_win_b"] = np.array(rec["b"], dtype=np.int64)
        out[f"{k}_win_seek"] = np.array(rec["seek"], dtype=np.int64)
        Lw = max(len(r_) for r_ in rec["ids"])
        out[f"{k}_win_ids"] = np.array([r_ + [-1] * (Lw - len(r_)) for r_ in rec["ids"]], dtype=np.int64)
        out[f"{k}_win_avg"] = np.array(rec["avg"], dtype=np.float64)
        out[f"{k}_win_ns"] = np.array(rec["ns"], dtype=np.float64)
        Ls = max(len(x) for x in rec["margin"])
        out[f"{k}_win_margin"] = np.stack([np.pad(x, (0, Ls - len(x)), constant_values=np.nan) for x in rec["margin"]])
        print(dims, "windows", list(zip(rec["b"], rec["seek"])), flush=True)
        del m


# ------------------------------------------------------------------------------------------------
# BASELINE-config parity fixtures (c1 / c2 / c3 dims).  The reference path is HF Whisper under
# bf16 autocast (run_distillation.py:815-830 mixed_precision="bf16"; accelerate wraps every prepared
# model's forward in autocast and upcasts its outputs to fp32, ACC accelerator.py:1818-1829), run here
# with torch.autocast("cpu", bfloat16): the same op policy for this model (Linear / Conv1d / SDPA in
# bf16 with fp32 accumulation, cross-entropy in fp32, LayerNorm statistics in fp32 -- CPU autocast
# returns LN of a bf16 stream in bf16 where CUDA returns fp32, identical once the next Linear casts
# it), the teacher's weights in bf16 (teacher_dtype, :1011-1018).  The fp32 model (mixed_precision
# "no") is stored beside it.


def _trainable(names, freeze_encoder, freeze_embed_positions):
    out = []
    for n in names:
        if n == "model.encoder.embed_positions.weight":
            continue
        if freeze_encoder and n.startswith("model.encoder."):
            continue
        if freeze_embed_positions and n == "model.decoder.embed_positions.weight":
            continue
        out.append(n)
    return out


def run_hf_step(S, T, feats, dec, lab, share, amp, temperature=2.0, amp_dtype=torch.bfloat16, scaler=None):
    """The reference train_step (run_distillation.py:1519-1551) on HF modules; returns scalars, the
    fp32 (upcast) logits and the encoder output; gradients land on S's parameters (loss-scaled when a
    GradScaler is given: accelerator.backward under mixed_precision="fp16" is scaler.scale(loss).backward())."""
    import contextlib
    from transformers.modeling_outputs import BaseModelOutput
    ctx = (lambda: torch.autocast("cpu", dtype=amp_dtype)) if amp else contextlib.nullcontext
    with ctx():
        so = S(input_features=feats, decoder_input_ids=dec, labels=lab)
    s_logits = so.logits.float()
    enc = so.encoder_last_hidden_state
    with torch.no_grad(), ctx():
        if share:
            to = T(encoder_outputs=BaseModelOutput(enc.detach().to(T.dtype)), labels=lab)
        else:
            to = T(input_features=feats, decoder_input_ids=dec, labels=lab)
    t_logits = to.logits.float()
    ce = so.loss.float()
    p = torch.softmax(t_logits / temperature, -1)
    lq = torch.log_softmax(s_logits / temperature, -1)
    mask = (lab >= 0).unsqueeze(-1)
    kl = (torch.nn.functional.kl_div(lq, p, reduction="none") * mask).sum() / mask.sum() * temperature ** 2
    loss = 0.8 * ce + kl
    (scaler.scale(loss) if scaler is not None else loss).backward()
    return dict(loss=loss.detach(), ce=ce.detach(), kl=kl.detach(), s_logits=s_logits.detach(),
                t_logits=t_logits.detach(), enc=enc.detach().float())


def gen_cfg(case, out):
    import time
    c = CFG_CASES[case]
    t0 = time.time()
    scfg, ws, tcfg, wt = cfg_case_weights(case)
    feats, dec, lab = cfg_case_batch(case)
    ft, dt, lt = torch.from_numpy(feats), torch.from_numpy(dec), torch.from_numpy(lab)
    share = c["freeze_encoder"] and scfg["d_model"] == tcfg["d_model"]
    out["dec"], out["lab"] = dec, lab
    out["share"] = np.array(share)
    print(case, "weights", round(time.time() - t0, 1), "s")
    for mode in ("f32", "amp"):
        S = hf_model(scfg, ws).train()
        T = hf_model(tcfg, wt, torch.bfloat16 if mode == "amp" else torch.float32).eval()
        names = [n for n, _ in S.named_parameters()]
        tr = _trainable(names, c["freeze_encoder"], c["freeze_embed_positions"])
        for n, p_ in S.named_parameters():
            p_.requires_grad_(n in tr)
        r = run_hf_step(S, T, ft, dt, lt, share, amp=(mode == "amp"))
        out[f"{mode}|loss"], out[f"{mode}|ce"], out[f"{mode}|kl"] = (np.float64(r[k].item())
                                                                     for k in ("loss", "ce", "kl"))
        out[f"{mode}|s_lse"] = torch.logsumexp(r["s_logits"], -1).numpy()
        out[f"{mode}|t_lse"] = torch.logsumexp(r["t_logits"], -1).numpy()
        out[f"{mode}|s_argmax"] = r["s_logits"].argmax(-1).numpy()
        out[f"{mode}|s_rows"] = r["s_logits"][:, ROWS, ::VSTRIDE].numpy()
        out[f"{mode}|enc_sub"] = r["enc"][:, ::50, :].numpy()
        out["grad_names"] = np.array(tr)
        out[f"{mode}|grad_norms"] = np.array([S.get_parameter(n).grad.double().norm().item() for n in tr])
        p0 = "model.decoder.layers.0.fc1.weight"
        out[f"{mode}|grad_dec0_fc1_sub"] = S.get_parameter(p0).grad[::37, ::29].clone().numpy()
        # clip + AdamW (lr 1e-4) as the sync micro-step applies them
        tp = [S.get_parameter(n) for n in tr]
        gn = torch.nn.utils.clip_grad_norm_(tp, 1.0)
        torch.optim.AdamW(tp, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0).step()
        out[f"{mode}|grad_total_norm"] = np.float64(gn.item())
        out[f"{mode}|upd_dec0_fc1_sub"] = S.get_parameter(p0).detach()[::37, ::29].clone().numpy()
        print(case, mode, {k: float(r[k]) for k in ("loss", "ce", "kl")}, round(time.time() - t0, 1), "s")
        del S, T, r


def gen_cfg_f16(case, out):
    """The fp16-autocast rows of a BASELINE-config fixture (mixed_precision="fp16", run_distillation.py:815-817):
    the student under torch.autocast(float16), the teacher's weights in fp16 (teacher_dtype), the loss through a
    default GradScaler (init scale 2^16; accelerate's fp16 path) -- unscale_ before the gradient norms and
    clip_grad_norm_, then scaler.step (AdamW) and scaler.update.  Keys "f16|..." merged into the existing file."""
    import time
    c = CFG_CASES[case]
    t0 = time.time()
    scfg, ws, tcfg, wt = cfg_case_weights(case)
    feats, dec, lab = cfg_case_batch(case)
    ft, dt, lt = torch.from_numpy(feats), torch.from_numpy(dec), torch.from_numpy(lab)
    share = c["freeze_encoder"] and scfg["d_model"] == tcfg["d_model"]
    S = hf_model(scfg, ws).train()
    T = hf_model(tcfg, wt, torch.float16).eval()
    tr = [n for n in out["grad_names"]]
    for n, p_ in S.named_parameters():
        p_.requires_grad_(n in tr)
    scaler = torch.amp.GradScaler("cpu")
    r = run_hf_step(S, T, ft, dt, lt, share, amp=True, amp_dtype=torch.float16, scaler=scaler)
    mode = "f16"
    out[f"{mode}|loss"], out[f"{mode}|ce"], out[f"{mode}|kl"] = (np.float64(r[k].item()) for k in ("loss", "ce", "kl"))
    out[f"{mode}|s_lse"] = torch.logsumexp(r["s_logits"], -1).numpy()
    out[f"{mode}|t_lse"] = torch.logsumexp(r["t_logits"], -1).numpy()
    out[f"{mode}|s_argmax"] = r["s_logits"].argmax(-1).numpy()
    out[f"{mode}|s_rows"] = r["s_logits"][:, ROWS, ::VSTRIDE].numpy()
    out[f"{mode}|enc_sub"] = r["enc"][:, ::50, :].numpy()
    tp = [S.get_parameter(n) for n in tr]
    opt = torch.optim.AdamW(tp, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
    out[f"{mode}|scale"] = np.float64(scaler.get_scale())
    scaler.unscale_(opt)
    out[f"{mode}|grad_norms"] = np.array([S.get_parameter(n).grad.double().norm().item() for n in tr])
    p0 = "model.decoder.layers.0.fc1.weight"
    out[f"{mode}|grad_dec0_fc1_sub"] = S.get_parameter(p0).grad[::37, ::29].clone().numpy()
    gn = torch.nn.utils.clip_grad_norm_(tp, 1.0)
    scaler.step(opt)
    scaler.update()
    out[f"{mode}|grad_total_norm"] = np.float64(gn.item())
    out[f"{mode}|scale_after"] = np.float64(scaler.get_scale())
    out[f"{mode}|upd_dec0_fc1_sub"] = S.get_parameter(p0).detach()[::37, ::29].clone().numpy()
    print(case, mode, {k: float(r[k]) for k in ("loss", "ce", "kl")}, "scale", scaler.get_scale(),
          round(time.time() - t0, 1), "s", flush=True)


def main():
    torch.manual_seed(0)
    only = sys.argv[1:]
    if only and only[0] == "f16":       # make_golden.py f16 c1 c2 ...: add the fp16-autocast rows to cfg fixtures
        for case in only[1:]:
            path = os.path.join(HERE, f"cfg_{case}.npz")
            z = np.load(path)
            out = {k: z[k] for k in z.files if not k.startswith("f16|")}
            gen_cfg_f16(case, out)
            np.savez_compressed(path, **out)
        return
    for name, fn in (("mel", gen_mel), ("mel_long", gen_mel_long), ("micro_step", gen_micro), ("student", gen_student), ("greedy", gen_greedy), ("beam", gen_beam), ("beam_ts", gen_beam_ts),
                     ("greedy_ts", gen_greedy_ts), ("fallback", gen_fallback), ("fp16", gen_fp16),
                     ("lv2_decode", gen_lv2_decode), ("batched_longform", gen_batched_longform),
                     ("cfg_c1", lambda o: gen_cfg("c1", o)), ("cfg_c2", lambda o: gen_cfg("c2", o)),
                     ("cfg_c3", lambda o: gen_cfg("c3", o)), ("cfg_c3b10", lambda o: gen_cfg("c3b10", o))):
        if only and name not in only:
            continue
        out = {}
        fn(out)
        if name == "lv2_decode" and os.environ.get("LV2_TAGS"):
            name = f"lv2_decode.{os.environ['LV2_TAGS'].replace(',', '_')}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, {k: getattr(v, "shape", None) for k, v in list(out.items())[:12]})


def lv2_merge():
    """Join the lv2_decode.<tags>.npz parts (LV2_TAGS runs) into lv2_decode.npz and remove them."""
    import glob
    out = {}
    parts = sorted(glob.glob(os.path.join(HERE, "lv2_decode.*.npz")))
    for p_ in parts:
        z = np.load(p_)
        out.update({k: z[k] for k in z.files})
    np.savez_compressed(os.path.join(HERE, "lv2_decode.npz"), **out)
    for p_ in parts:
        os.remove(p_)
    print("lv2_decode", sorted(out))


if __name__ == "__main__":
    if sys.argv[1:] == ["lv2_merge"]:
        lv2_merge()
    else:
        main()
