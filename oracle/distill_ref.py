"""ORACLE (test infrastructure only): restatement of the distillation step.

Reference: `training/run_distillation.py`
  kl_divergence        :1507-1516  KLDivLoss(reduction="none")(log q, p), masked by
                                   labels >= 0, summed, / count(labels >= 0)
  train_step           :1519-1551  student(**batch); no_grad teacher (shared frozen
                                   encoder -> teacher(encoder_outputs=enc.to(bf16),
                                   labels=labels), i.e. decoder input =
                                   shift_tokens_right(labels)); p = softmax(t/T),
                                   log q = log_softmax(s/T); kl * T^2;
                                   loss = 0.8 * ce + kl_weight * kl
  eval_step            :1554-1578  same with T = 1 and no grad
  optimizer groups     :1425-1455  decay = non-LayerNorm, non-bias names outside
                                   frozen modules (get_parameter_names :777-795)
  clip + AdamW         :1666-1668  clip_grad_norm_(max_grad_norm) then
                                   torch.optim.AdamW(betas, eps) step (the
                                   reference's own optimizer is used directly here)
  lr schedule          :1458-1463  constant_with_warmup, warmup * N and stepped N
                                   times per update (Accelerate) == per-update warmup
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .whisper_ref import Ref


def kl_divergence(target_distribution, log_predicted_distribution, labels):
    div = F.kl_div(log_predicted_distribution, target_distribution, reduction="none")
    mask = (labels >= 0).unsqueeze(-1)
    div = div * mask
    return div.sum() / mask.sum()


def distill_loss(s_logits, t_logits, labels, ce, temperature=2.0, kl_weight=1.0):
    p = F.softmax(t_logits / temperature, dim=-1)
    logq = F.log_softmax(s_logits / temperature, dim=-1)
    kl = kl_divergence(p, logq, labels) * temperature ** 2
    loss = 0.8 * ce + kl_weight * kl
    return loss, kl


def train_step(student: Ref, teacher: Ref, feats, decoder_input_ids, labels, temperature=2.0,
               kl_weight=1.0, share_hidden_states=True):
    """Returns dict(loss, ce_loss, kl_loss); grads land on student params' .grad."""
    s = student.forward(feats, decoder_input_ids, labels)
    with torch.no_grad():
        if share_hidden_states:
            enc = s["enc"].detach()
            if teacher.sbf:
                enc = enc.to(torch.bfloat16).float()
            t = teacher.forward(enc=enc, labels=labels)
        else:
            t = teacher.forward(feats, decoder_input_ids, labels)
    loss, kl = distill_loss(s["logits"], t["logits"], labels, s["loss"], temperature, kl_weight)
    loss.backward()
    return dict(loss=loss.detach(), ce_loss=s["loss"].detach(), kl_loss=kl.detach(),
                s_logits=s["logits"].detach(), t_logits=t["logits"].detach())


def eval_step(student: Ref, teacher: Ref, feats, decoder_input_ids, labels, kl_weight=1.0,
              share_hidden_states=True):
    with torch.no_grad():
        s = student.forward(feats, decoder_input_ids, labels)
        if share_hidden_states:
            enc = s["enc"].to(torch.bfloat16).float() if teacher.sbf else s["enc"]
            t = teacher.forward(enc=enc, labels=labels)
        else:
            t = teacher.forward(feats, decoder_input_ids, labels)
        p = F.softmax(t["logits"], -1)
        logq = F.log_softmax(s["logits"], -1)
        kl = kl_divergence(p, logq, labels)
        return dict(loss=0.8 * s["loss"] + kl_weight * kl, ce_loss=s["loss"], kl_loss=kl)


def decay_parameter_names(names, frozen_prefixes=()):
    """get_parameter_names(student, [nn.LayerNorm], forbidden_module) minus 'bias'."""
    out = []
    for n in names:
        if any(n.startswith(f) for f in frozen_prefixes):
            continue
        if "layer_norm" in n or "bias" in n:
            continue
        out.append(n)
    return out


def constant_with_warmup(step: int, warmup: int) -> float:
    """LR multiplier after `step` optimizer updates (HF get_constant_schedule_with_warmup,
    with Accelerate's N-fold warmup and N-fold stepping cancelling)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return 1.0


def optimizer_step(params: dict, trainable, lr, weight_decay=0.0, betas=(0.9, 0.999), eps=1e-8,
                   max_grad_norm=1.0, state=None, frozen_prefixes=()):
    """clip_grad_norm_ + torch.optim.AdamW step over `trainable` names (grads on .grad).
    Returns (grad_norm, optimizer)."""
    tp = [params[n] for n in trainable]
    gn = torch.nn.utils.clip_grad_norm_(tp, max_grad_norm)
    decay = set(decay_parameter_names(trainable, frozen_prefixes))
    if state is None:
        state = torch.optim.AdamW(
            [dict(params=[params[n] for n in trainable if n in decay], weight_decay=weight_decay),
             dict(params=[params[n] for n in trainable if n not in decay], weight_decay=0.0)],
            lr=lr, betas=betas, eps=eps, foreach=False)
    for g in state.param_groups:
        g["lr"] = lr
    state.step()
    return gn, state
