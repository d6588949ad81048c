"""Checkpoint / resume in the reference's layout.

Reference: `training/run_distillation.py` —
  * `sorted_checkpoints` / `rotate_checkpoints` / `get_last_checkpoint` (:730-774): directories
    `checkpoint-{step}-epoch-{epoch}` under output_dir, oldest deleted beyond save_total_limit;
  * save (:1685-1699): `accelerator.save_state(output_dir/checkpoint-{step}-epoch-{epoch})`;
  * resume (:1607-1640): `accelerator.load_state(dir)`, step/epoch parsed from the name, the
    dataloader skipped by `(cur_step - epochs_trained * steps_per_epoch) * accum` batches when the
    epoch length is known (else one extra shuffle, fresh epoch);
  * final (:1814-1818): `save_pretrained(output_dir)`.
Accelerate's `save_state` directory (accelerate/checkpointing.py): `model.safetensors` (student),
`model_1.safetensors` (teacher, prepared second at :1503), `optimizer.bin` / `scheduler.bin`
(torch.save of the torch AdamW / LambdaLR state dicts), `random_states_{rank}.pkl`.

The optimizer state dict follows torch.optim.AdamW's format over the reference's parameter
groups (:1434-1456): group 0 = the student's HF `named_parameters()` (tied proj_out de-duplicated)
that `get_parameter_names(student, [LayerNorm], forbidden_module=[frozen encoder/decoder])` keeps
and whose name has no "bias"; group 1 = every other parameter (frozen ones included, they only
carry no state).  Indices run over group 0 then group 1, so a checkpoint written here loads into
the reference's optimizer and vice versa.
"""
from __future__ import annotations

import os
import re
import shutil
from pathlib import Path
from typing import List, Optional, Tuple

CHECKPOINT_RE = re.compile(r"^checkpoint-(\d+)-epoch-(\d+)$")


def checkpoint_name(step: int, epoch: int) -> str:
    return f"checkpoint-{step}-epoch-{epoch}"


def sorted_checkpoints(output_dir, checkpoint_prefix: str = "checkpoint") -> List[str]:
    """Checkpoint directories under output_dir, oldest (smallest step) first."""
    found = []
    for p in Path(output_dir).glob(f"{checkpoint_prefix}-*"):
        if not p.is_dir():
            continue
        m = re.match(rf".*{checkpoint_prefix}-([0-9]+)", str(p))
        if m:
            found.append((int(m.group(1)), str(p)))
    return [p for _, p in sorted(found)]


def rotate_checkpoints(save_total_limit: Optional[int], output_dir, checkpoint_prefix: str = "checkpoint") -> List[str]:
    """Delete the oldest checkpoints beyond save_total_limit; returns the deleted paths."""
    if save_total_limit is None or save_total_limit <= 0:
        return []
    ck = sorted_checkpoints(output_dir, checkpoint_prefix)
    if len(ck) <= save_total_limit:
        return []
    doomed = ck[: len(ck) - save_total_limit]
    for p in doomed:
        shutil.rmtree(p, ignore_errors=True)
    return doomed


def get_last_checkpoint(folder) -> Optional[str]:
    names = [n for n in os.listdir(folder) if CHECKPOINT_RE.search(n) and os.path.isdir(os.path.join(folder, n))]
    if not names:
        return None
    return os.path.join(folder, max(names, key=lambda n: int(CHECKPOINT_RE.search(n).group(1))))


def parse_checkpoint(path: str) -> Tuple[int, int]:
    m = re.search(r"checkpoint-(\d+)-epoch-(\d+)", path)
    if m is None:
        raise ValueError(f"not a checkpoint-{{step}}-epoch-{{epoch}} path: {path}")
    return int(m.group(1)), int(m.group(2))


def resume_skip_batches(cur_step: int, epochs_trained: int, steps_per_epoch: Optional[int], accum: int,
                        streaming: bool, max_steps: int) -> Optional[int]:
    """Batches to skip in the resumed epoch (run_distillation.py:1629-1636); None = the reference's
    "unknown epoch length" path (shuffle once more and start a fresh epoch)."""
    if not streaming and max_steps < 0 and steps_per_epoch:
        return (cur_step - epochs_trained * steps_per_epoch) * accum
    return None


def hf_parameter_names(cfg) -> List[str]:
    """HF WhisperForConditionalGeneration.named_parameters() order (module registration order:
    encoder conv1, conv2, embed_positions, layers[k_proj, v_proj, q_proj, out_proj, LN, fc1, fc2,
    final LN], layer_norm; decoder embed_tokens, embed_positions, layers[self attn, LN, cross
    attn, LN, fc1, fc2, final LN], layer_norm; proj_out tied -> de-duplicated)."""
    names = []
    e, d = "model.encoder", "model.decoder"

    def attn(p):
        return [f"{p}.k_proj.weight", f"{p}.v_proj.weight", f"{p}.v_proj.bias", f"{p}.q_proj.weight",
                f"{p}.q_proj.bias", f"{p}.out_proj.weight", f"{p}.out_proj.bias"]

    def ln(p):
        return [f"{p}.weight", f"{p}.bias"]

    def mlp(p):
        return [f"{p}.fc1.weight", f"{p}.fc1.bias", f"{p}.fc2.weight", f"{p}.fc2.bias"] + ln(f"{p}.final_layer_norm")

    names += [f"{e}.conv1.weight", f"{e}.conv1.bias", f"{e}.conv2.weight", f"{e}.conv2.bias",
              f"{e}.embed_positions.weight"]
    for i in range(cfg.encoder_layers):
        p = f"{e}.layers.{i}"
        names += attn(p + ".self_attn") + ln(p + ".self_attn_layer_norm") + mlp(p)
    names += ln(f"{e}.layer_norm")
    names += [f"{d}.embed_tokens.weight", f"{d}.embed_positions.weight"]
    for i in range(cfg.decoder_layers):
        p = f"{d}.layers.{i}"
        names += attn(p + ".self_attn") + ln(p + ".self_attn_layer_norm")
        names += attn(p + ".encoder_attn") + ln(p + ".encoder_attn_layer_norm") + mlp(p)
    names += ln(f"{d}.layer_norm")
    return names


def optimizer_groups(cfg, freeze_encoder: bool, freeze_decoder: bool) -> Tuple[List[str], List[str]]:
    """(decay names, other names) in the reference's group order (:1424-1449)."""
    forbidden = [p for p, f in (("model.encoder.", freeze_encoder), ("model.decoder.", freeze_decoder)) if f]
    names = hf_parameter_names(cfg)

    def decays(n):
        return not any(n.startswith(f) for f in forbidden) and "layer_norm" not in n and "bias" not in n

    return [n for n in names if decays(n)], [n for n in names if not decays(n)]
