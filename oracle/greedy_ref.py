"""ORACLE (test infrastructure only): greedy decode restatement.

Reference decode calls: `training/run_distillation.py:1580-1584` (generate_step),
`training/run_pseudo_labelling.py:917-922` (`generate(num_beams=1, language, task)`),
`pseudo-labelling/initial_inference.py:36-41` (faster-whisper; unpinned and absent,
SURVEY.md finding 10 -> parity pinned to HF greedy generate).

HF Whisper generate (HF:generation_whisper.py) with language/task and no timestamps:
prompt [SOT, lang, task, <|notimestamps|>]; per step logits of the last position,
SuppressTokens (generation_config.suppress_tokens) every step, SuppressTokensAtBegin
([220, eos]) at the first generated step (HF:generation/logits_process.py), argmax,
stop at eos or max_length.  This oracle recomputes the whole prefix each step (no
cache) so it shares nothing with the KV-cache path it checks.
"""
from __future__ import annotations

import torch

from .whisper_ref import Ref


def greedy(model: Ref, feats, prompt, max_length=448, suppress_tokens=(), begin_suppress=(220, 50257),
           eos=50257, return_scores=False):
    enc = model.encoder(feats)
    B = feats.shape[0]
    ids = torch.tensor(prompt, dtype=torch.long).unsqueeze(0).repeat(B, 1)
    done = torch.zeros(B, dtype=torch.bool)
    scores = []
    while ids.shape[1] < max_length:
        h = model.decoder(ids, enc)
        lg = model.logits(h[:, -1:])[:, 0].clone()
        if len(suppress_tokens):
            lg[:, list(suppress_tokens)] = float("-inf")
        if ids.shape[1] == len(prompt) and len(begin_suppress):
            lg[:, list(begin_suppress)] = float("-inf")
        scores.append(lg)
        nxt = lg.argmax(-1)
        nxt = torch.where(done, torch.full_like(nxt, eos), nxt)
        ids = torch.cat([ids, nxt[:, None]], 1)
        done |= nxt == eos
        if bool(done.all()):
            break
    return (ids, scores) if return_scores else ids
