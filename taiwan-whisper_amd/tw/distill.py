"""The distillation step — MI355X-native counterpart of the closures in
`training/run_distillation.py`:

  kl_divergence / train_step / eval_step   :1507-1578
  freezing + share_hidden_states           :1043-1075
  optimizer groups / AdamW / scheduler     :1425-1463 (weight decay on non-LN, non-bias names)
  accumulate / backward / clip / step      :1662-1670 (Accelerate: loss / accum, DDP mean over ranks)

Everything runs on the GPU through libtw_hip.so; nothing on the step synchronises with the host
(metrics stay device tensors until the caller reads them).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import ops as F
from .modeling import Backward, WhisperForConditionalGeneration, is_pseudo


def constant_with_warmup(step: int, warmup: int) -> float:
    """HF get_constant_schedule_with_warmup as Accelerate drives it (warmup*N, stepped N times per
    update): update k uses lr * min(1, k / warmup)."""
    if warmup > 0 and step < warmup:
        return step / warmup
    return 1.0


def linear_schedule(step: int, warmup: int, total: int) -> float:
    if warmup > 0 and step < warmup:
        return step / warmup
    return max(0.0, (total - step) / max(1, total - warmup))


def set_trainable_like_reference(student: WhisperForConditionalGeneration, freeze_encoder: bool,
                                 freeze_decoder: bool, freeze_embed_positions: bool):
    """The trainable set of run_distillation.py:1043-1066 (HF keeps encoder.embed_positions frozen;
    with freeze_decoder the tied proj_out = embed_tokens stays trainable)."""
    student.set_trainable("", True)
    student.set_trainable("model.encoder.embed_positions", False)
    if freeze_encoder:
        student.set_trainable("model.encoder", False)
    if freeze_decoder:
        student.set_trainable("model.decoder", False)
        student.set_trainable("model.decoder.embed_tokens", True)
    if freeze_embed_positions:
        student.set_trainable("model.decoder.embed_positions", False)
    return student


def weight_decay_runs(s: WhisperForConditionalGeneration, wd: float, freeze_encoder: bool, freeze_decoder: bool):
    """Maximal [lo, hi) ranges of the packed trainable prefix sharing one weight decay.  The decay set is
    the reference's group 0 (run_distillation.py:1424-1449: get_parameter_names(student, [LayerNorm],
    forbidden_module=[frozen encoder / decoder]) minus "bias" names) -- the same rule
    tw/checkpoint.optimizer_groups writes into optimizer.bin, so with freeze_decoder the trainable
    embed_tokens (under the frozen decoder module) is NOT decayed."""
    from .checkpoint import optimizer_groups
    decay = set(optimizer_groups(s.config, freeze_encoder, freeze_decoder)[0])
    runs = []
    for n in s.train_names:
        w = wd if n in decay else 0.0          # the pseudo k_proj.zero_bias segments are never decayed
        lo = s.store.offset[n]
        hi = (lo + s.store.numel(n) + 63) // 64 * 64
        if runs and runs[-1][2] == w and runs[-1][1] == lo:
            runs[-1][1] = hi
        else:
            runs.append([lo, hi, w])
    return [tuple(r) for r in runs]


class GradScaler:
    """torch.amp.GradScaler as accelerate builds it for mixed_precision="fp16" (run_distillation.py:815-827; ACC
    accelerator.py: GradScaler(**kwargs) with the defaults): the loss gradient is multiplied by `scale`; at the sync
    micro-step a non-finite gradient norm skips the optimizer step (and, in accelerate, the scheduler step) and halves
    the scale, else the step runs on gradient / scale and after `growth_interval` finite steps in a row the scale
    doubles.  Host-side state: the engine reads the norm once per update to decide (torch's GradScaler.step reads
    found_inf the same way)."""

    def __init__(self, init_scale=65536.0, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        self.scale = float(init_scale)
        self.growth_factor, self.backoff_factor = float(growth_factor), float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.growth_tracker = 0

    def update(self, found_inf: bool):
        """GradScaler.update (torch _amp_update_scale_)."""
        if found_inf:
            self.scale *= self.backoff_factor
            self.growth_tracker = 0
        else:
            self.growth_tracker += 1
            if self.growth_tracker == self.growth_interval:
                self.scale *= self.growth_factor
                self.growth_tracker = 0

    def state_dict(self):
        return {"scale": self.scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self.growth_tracker}

    def load_state_dict(self, sd):
        self.scale = float(sd["scale"])
        self.growth_factor, self.backoff_factor = float(sd["growth_factor"]), float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
        self.growth_tracker = int(sd["_growth_tracker"])


class DistillationTrainer:
    def __init__(self, student: WhisperForConditionalGeneration, teacher: WhisperForConditionalGeneration, *,
                 temperature: float = 2.0, kl_weight: float = 1.0, learning_rate: float = 1e-4,
                 adam_beta1: float = 0.9, adam_beta2: float = 0.999, adam_epsilon: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0, warmup_steps: int = 0,
                 lr_scheduler_type: str = "constant_with_warmup", max_steps: int = 0,
                 gradient_accumulation_steps: int = 1, freeze_encoder: bool = True, freeze_decoder: bool = False,
                 freeze_embed_positions: bool = True, process_group=None, dp_bucket_mb: int = 64,
                 overlap_update: Optional[bool] = None, force_exchange: bool = False):
        if student.compute != teacher.compute:
            raise ValueError(f"student computes in {student.compute}, teacher in {teacher.compute}: the reference "
                             "runs both under one mixed_precision setting")
        self.s, self.t = student, teacher
        self.temperature, self.kl_weight = temperature, kl_weight
        self.lr, self.b1, self.b2, self.eps = learning_rate, adam_beta1, adam_beta2, adam_epsilon
        self.wd, self.max_grad_norm = weight_decay, max_grad_norm
        self.warmup, self.sched, self.max_steps = warmup_steps, lr_scheduler_type, max_steps
        self.accum = gradient_accumulation_steps
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        # force_exchange (tests, bench rehearsal): run the whole DP exchange -- per-layer async all-reduces from the
        # backward hook, the tail, the waits, the deferred update -- even on a process group of ONE rank, so the
        # RCCL code path executes on a 1-GPU box (an all-reduce over one rank is the identity: bit-identical)
        self.force_exchange = bool(force_exchange) and process_group is not None
        self.dp = self.world > 1 or self.force_exchange
        self.bucket = dp_bucket_mb * (1 << 20) // 4
        # DDP mean (torch Reducer, no comm hook): every rank's gradient is multiplied by fp32(1/world) as it
        # enters its bucket, then the buckets are SUM-all-reduced.  For a power-of-two world the factor is
        # exact and commutes with every rounding of the backward, so it is folded into the loss gradient
        # (no extra pass); otherwise each slice is scaled right before its all-reduce, as DDP does.
        self.fold_world = self.world & (self.world - 1) == 0
        # Deferred update (DP, frozen encoder): the gradient exchange of the sync micro-step is launched at
        # its end, but the wait + clip + AdamW are queued only after the NEXT step's encoder forward, which
        # reads no trainable weight.  The exchange of the last-finished gradients (the tied embedding,
        # 265 MB at c3, final only after the embedding backward) then runs beside that encoder instead of
        # stalling the stream.  Same kernels on the same data in the same order per buffer: bit-identical.
        # Any reader of the weights or optimizer state (eval, state dicts, save) calls flush() first.
        self.overlap_update = (self.dp and freeze_encoder) if overlap_update is None else bool(overlap_update)
        if self.overlap_update and not freeze_encoder:
            raise ValueError("overlap_update needs a frozen encoder: the next forward must read no trainable weight")
        # fp16 autocast (--dtype float16): dynamic loss scaling.  Whether an update runs depends on the norm of the
        # exchanged gradient, read on the host at the sync micro-step, so the update is never deferred.
        self.scaler = GradScaler() if student.compute == "fp16" else None
        if self.scaler is not None:
            if student.dtype != torch.float32:
                raise ValueError("fp16 distillation trains an fp32-master student under fp16 autocast")
            if overlap_update:
                raise ValueError("overlap_update: the fp16 loss scaler decides each update on the host")
            self.overlap_update = False
        self.skipped_steps = 0   # fp16: optimizer steps skipped for a non-finite gradient (GradScaler)
        self._update = None      # (lr, t) of a launched, not yet applied update
        # bench.py instrumentation: with lists here, wait_grad_exchange() appends (start, layers done, tail done)
        # events around each exchange wait and _launch() appends (bytes, tail) per all-reduced slice
        self.exchange_events = None
        self.exchange_log = None
        set_trainable_like_reference(student, freeze_encoder, freeze_decoder, freeze_embed_positions)
        self.train_encoder = not freeze_encoder
        self.freeze_encoder, self.freeze_decoder = freeze_encoder, freeze_decoder
        self.share = freeze_encoder and student.config.d_model == teacher.config.d_model
        student.pack_for_training()
        student.sync_bf16()
        student.train()
        teacher.eval()
        n = student.train_prefix
        self.m_buf = torch.zeros(n, dtype=torch.float32, device=student.device)
        self.v_buf = torch.zeros(n, dtype=torch.float32, device=student.device)
        self.norm = torch.zeros(1, dtype=torch.float32, device=student.device)
        self.ws = torch.zeros(1024, dtype=torch.float32, device=student.device)
        self.nvalid = torch.zeros(1, dtype=torch.int32, device=student.device)
        self.step = 0            # completed optimizer updates
        self.micro = 0
        self.bw = Backward(student)
        self.runs = self._wd_runs()

    def _wd_runs(self):
        return weight_decay_runs(self.s, self.wd, self.freeze_encoder, self.freeze_decoder)

    def num_trainable_parameters(self):
        return self.s.num_parameters(only_trainable=True)

    def lr_at(self, step):
        if self.sched == "linear":
            return self.lr * linear_schedule(step, self.warmup, self.max_steps)
        if self.sched == "constant":
            return self.lr
        return self.lr * constant_with_warmup(step, self.warmup)

    # ------------------------------------------------------------------ forward pieces
    def _conv_input(self, batch):
        ci = batch.get("conv_input")
        if ci is not None and ci.dtype == self.s.act_dtype:
            return ci                       # the feed's log-mel kernel emitted it in the compute dtype
        return self.s.conv_input(batch["input_features"])

    def _teacher_logits(self, conv_in, ids, labels, enc16, Tk):
        t = self.t
        if self.share:
            t_ids = torch.empty_like(labels)
            F.shift_tokens_right(labels, t_ids, t.config.pad_token_id, t.config.decoder_start_token_id)
            ht = t.decode(t_ids, enc16, Tk)
        else:
            enc_t = t.encode(conv_in)
            ht = t.decode(ids, enc_t, Tk)
        return t.lm_head(ht)

    def train_step(self, batch, temperature: Optional[float] = None, end_of_dataloader: bool = False):
        """One micro-step: student fwd + teacher fwd + fused KL/CE + backward (+ DP exchange,
        clip and AdamW on the sync micro-step).  Returns device scalars.

        Sync micro-step = every `accum`-th one, or the last batch of the dataloader (accelerate's
        GradientState syncs at end_of_dataloader and restarts its count, ACC accelerator.py _do_sync):
        the partial accumulation -- k < accum gradients, each already scaled by 1/accum -- is applied."""
        T = self.temperature if temperature is None else temperature
        s = self.s
        conv_in = self._conv_input(batch)
        ids = batch["decoder_input_ids"].to(s.device).contiguous()
        labels = batch["labels"].to(s.device).contiguous()
        B, Td = ids.shape
        enc_tape = [] if self.train_encoder else None
        enc16 = s.encode(conv_in, tape=enc_tape)
        self.flush()             # the previous update (its exchange ran beside the encoder above)
        if self.micro == 0:
            s.grad.zero_()
        # DP: on the micro-step that syncs, each layer's gradient slice is all-reduced as soon as
        # the backward has finished it (RCCL on its own stream, beside the remaining backward)
        self._pending, self._reduced = [], []
        sync = self.micro + 1 == self.accum or end_of_dataloader
        self.bw.on_ready = self._grad_ready if (self.dp and sync) else None
        Tk = enc16.shape[0] // B
        tape = []
        hs = s.decode(ids, enc16, Tk, tape=tape)
        ls = s.lm_head(hs)
        with torch.no_grad():
            lt = self._teacher_logits(conv_in, ids, labels, enc16, Tk)
        lab = labels.reshape(-1)
        F.count_valid(lab, self.nvalid)
        dlogits = ls      # the loss gradient overwrites the student logits in place (tw_kl_ce): one [B*T, V] block less
        # the loss gradient: 1 / accum (accelerate's backward), the folded DDP mean, and fp16's loss scale
        # (scaler.scale(loss).backward(): the scale enters the fp32 gradient before its fp16 rounding)
        gs = (self.scaler.scale if self.scaler is not None else 1.0) / (self.accum * (self.world if self.fold_world
                                                                                         else 1))
        out3, _ = F.kl_ce(ls, lt, lab, s.config.vocab_size, self.nvalid, T=T, ce_w=0.8, kl_w=self.kl_weight,
                          grad_scale=gs, dlogits=dlogits)
        del lt
        d_enc = torch.zeros(B * Tk, s.config.d_model, dtype=torch.float32, device=s.device) \
            if self.train_encoder else None
        self.bw.decoder(tape, dlogits, hs, enc16, d_enc)
        del tape, dlogits, ls
        if self.train_encoder:
            self.bw.encoder(enc_tape, d_enc)
        self.micro += 1
        if sync:
            self.optimizer_step()
            self.micro = 0
        return {"loss": out3[0], "ce_loss": out3[1], "kl_loss": out3[2]}

    def eval_step(self, batch):
        """run_distillation.py:1554-1578: T = 1, no grad."""
        self.flush()
        s = self.s
        conv_in = self._conv_input(batch)
        ids = batch["decoder_input_ids"].to(s.device).contiguous()
        labels = batch["labels"].to(s.device).contiguous()
        B = ids.shape[0]
        enc16 = s.encode(conv_in)
        Tk = enc16.shape[0] // B
        ls = s.lm_head(s.decode(ids, enc16, Tk))
        lt = self._teacher_logits(conv_in, ids, labels, enc16, Tk)
        lab = labels.reshape(-1)
        nv = torch.zeros(1, dtype=torch.int32, device=s.device)
        F.count_valid(lab, nv)
        out3, _ = F.kl_ce(ls, lt, lab, s.config.vocab_size, nv, T=1.0, ce_w=0.8, kl_w=self.kl_weight)
        return {"loss": out3[0], "ce_loss": out3[1], "kl_loss": out3[2]}

    # ------------------------------------------------------------------ update
    def _launch(self, lo, hi, tail=False):
        """Async SUM all-reduce of grad[lo:hi) in buckets.  tail: launched after the backward (the ranges no
        layer hook covered: the embeddings, the final LayerNorm), i.e. the part that cannot overlap it."""
        g = self.s.grad
        for a in range(lo, hi, self.bucket):
            sl = g[a: min(hi, a + self.bucket)]
            if not self.fold_world:
                sl.mul_(1.0 / self.world)          # DDP: grad * fp32(1/world) into the bucket, then SUM
            self._pending.append((torch.distributed.all_reduce(sl, group=self.pg, async_op=True), tail))
            if getattr(self, "exchange_log", None) is not None:
                self.exchange_log.append((sl.numel() * sl.element_size(), tail))
        self._reduced.append((lo, hi))

    def _grad_ready(self, prefix):
        r = self.s.grad_range(prefix)
        if r is not None:
            self._launch(*r)

    def launch_grad_exchange(self):
        """Launch the part of the DDP-mean exchange not yet started: ranges whose exchange began during
        the backward (per finished layer) are skipped; the rest (embeddings, final LayerNorm, ...) is
        launched now.  Bucketed async SUM all-reduce of the flat fp32 gradient over RCCL, each rank's
        gradient scaled by 1/world first (folded into the loss gradient for power-of-two worlds)."""
        if not self.dp:
            return
        done = sorted(getattr(self, "_reduced", []))
        pos = 0
        if not hasattr(self, "_pending"):
            self._pending = []
        for lo, hi in done + [(self.s.grad.numel(), self.s.grad.numel())]:
            if lo > pos:
                self._launch(pos, lo, tail=True)
            pos = max(pos, hi)
        self._reduced = []
        self.bw.on_ready = None

    def wait_grad_exchange(self):
        """The compute stream waits for every launched bucket (a stream dependency under RCCL).  With
        `exchange_events` a list (bench.py), events bracket the wait on the compute stream: first the buckets
        launched during the backward (per finished layer), then the tail launched after it (the tied embedding,
        final LayerNorm).  Their distances are the exchange time the step leaves exposed, split into the two."""
        pend = getattr(self, "_pending", [])
        ev = getattr(self, "exchange_events", None) if pend else None
        if ev is not None:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
        for w, tail in pend:            # RCCL runs them in launch order: layers first, then the tail
            if not tail:
                w.wait()
        if ev is not None:
            e[1].record()
        for w, tail in pend:
            if tail:
                w.wait()
        if ev is not None:
            e[2].record()
            ev.append(tuple(e))
        self._pending, self._reduced = [], []

    def all_reduce_grads(self):
        """DDP mean over ranks: launch what is left of the exchange, then wait for all of it."""
        self.launch_grad_exchange()
        self.wait_grad_exchange()

    def _apply_update(self, lr, t):
        """Clip + AdamW; returns False when the fp16 loss scaler skipped the step (non-finite gradient norm)."""
        s = self.s
        self.wait_grad_exchange()
        g = s.grad
        F.l2norm(g, self.norm, self.ws)
        inv = 1.0
        if self.scaler is not None:
            # GradScaler.unscale_ + clip_grad_norm_ + step: the norm of the scaled gradient is finite iff every
            # element is (up to an fp32 overflow of the sum of squares); unscaling by a power of two is exact, so
            # adamw_ex applies g / scale and norm / scale inside the update kernel
            found_inf = not math.isfinite(float(self.norm.item()))
            scale = self.scaler.scale
            self.scaler.update(found_inf)
            if found_inf:
                self.skipped_steps += 1
                return False
            inv = 1.0 / scale
        for lo, hi, wd in self.runs:
            F.adamw(s.store.p32[lo:hi], g[lo:hi], self.m_buf[lo:hi], self.v_buf[lo:hi], s.store.p16[lo:hi], lr,
                    self.b1, self.b2, self.eps, wd, t, self.norm, self.max_grad_norm, inv_scale=inv)
        return True

    def optimizer_step(self):
        """Clip + AdamW on the exchanged gradient.  With overlap_update the exchange is launched here and the
        update is applied by the next flush() (the next train_step, after its encoder forward); `self.norm`
        holds the clipped-over norm once it has run."""
        lr, t = self.lr_at(self.step), self.step + 1
        self.launch_grad_exchange()
        if self.overlap_update:
            self.step += 1
            self._update = (lr, t)
        elif self._apply_update(lr, t):
            self.step += 1     # a skipped fp16 step leaves AdamW's step count and the schedule where they were
        return self.norm

    def flush(self):
        """Apply a deferred update (no-op without one).  Call before reading weights or optimizer state."""
        if self._update is not None:
            lr, t = self._update
            self._update = None
            self._apply_update(lr, t)

    # ------------------------------------------------------------------ checkpoint state
    def state_dict(self):
        self.flush()
        return {"step": self.step, "exp_avg": self.m_buf, "exp_avg_sq": self.v_buf}

    def load_state_dict(self, st):
        self.flush()
        self.step = int(st["step"])
        self.m_buf.copy_(st["exp_avg"])
        self.v_buf.copy_(st["exp_avg_sq"])

    def _moment_view(self, buf, n):
        """HF-shaped view of a trainable segment of a flat moment buffer (engine layout)."""
        from .modeling import to_hf
        s = self.s
        o = s.store.offset[n]
        return to_hf(n, buf[o: o + s.store.numel(n)].view(s.store.segs[n]), s.config)

    def optimizer_state_dict(self):
        """torch.optim.AdamW.state_dict() of the reference's optimizer (tw/checkpoint.py groups)."""
        self.flush()
        from .checkpoint import optimizer_groups
        g0, g1 = optimizer_groups(self.s.config, self.freeze_encoder, self.freeze_decoder)
        state, idx = {}, 0
        groups = []
        lr = self.lr_at(self.step)
        for names, wd in ((g0, self.wd), (g1, 0.0)):
            ids = []
            for n in names:
                if n in self.s.trainable and self.step > 0:
                    state[idx] = {"step": torch.tensor(float(self.step)),
                                  "exp_avg": self._moment_view(self.m_buf, n).detach().cpu().clone(),
                                  "exp_avg_sq": self._moment_view(self.v_buf, n).detach().cpu().clone()}
                ids.append(idx)
                idx += 1
            groups.append({"lr": lr, "betas": (self.b1, self.b2), "eps": self.eps, "weight_decay": wd,
                           "amsgrad": False, "foreach": None, "maximize": False, "capturable": False,
                           "differentiable": False, "fused": None, "decoupled_weight_decay": True,
                           "initial_lr": self.lr, "params": ids})
        return {"state": state, "param_groups": groups}

    def load_optimizer_state_dict(self, sd):
        """Inverse of optimizer_state_dict (also accepts the reference's own optimizer.bin)."""
        self.flush()
        from .checkpoint import optimizer_groups
        g0, g1 = optimizer_groups(self.s.config, self.freeze_encoder, self.freeze_decoder)
        order = g0 + g1
        if len(order) != sum(len(g["params"]) for g in sd["param_groups"]):
            raise ValueError("optimizer state: parameter count differs from the reference grouping")
        flat = [i for g in sd["param_groups"] for i in g["params"]]
        steps = set()
        self.m_buf.zero_()
        self.v_buf.zero_()
        for n, i in zip(order, flat):
            st = sd["state"].get(i)
            if st is None:
                continue
            if n not in self.s.trainable:
                raise ValueError(f"optimizer state for {n}, which is frozen here")
            self._moment_view(self.m_buf, n).copy_(st["exp_avg"])
            self._moment_view(self.v_buf, n).copy_(st["exp_avg_sq"])
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"optimizer state: mixed step counts {sorted(steps)}")
        self.step = steps.pop() if steps else 0

    def scheduler_state_dict(self):
        """LambdaLR.state_dict() of get_scheduler(...) stepped world times per update (:1458-1463)."""
        n = self.step * self.world
        return {"base_lrs": [self.lr, self.lr], "last_epoch": n, "verbose": False, "_step_count": n + 1,
                "_get_lr_called_within_step": False, "_last_lr": [self.lr_at(self.step)] * 2,
                "lr_lambdas": [None, None]}

    def save_state(self, output_dir, save_teacher=True, rank=0):
        """accelerator.save_state layout (tw/checkpoint.py)."""
        self.flush()
        from safetensors.torch import save_file
        os.makedirs(output_dir, exist_ok=True)
        if rank == 0:
            for i, m in enumerate([self.s] + ([self.t] if save_teacher else [])):
                sd = {k: v.detach().to("cpu").contiguous() for k, v in m.state_dict().items() if k != "proj_out.weight"}
                save_file(sd, os.path.join(output_dir, "model.safetensors" if i == 0 else f"model_{i}.safetensors"),
                          metadata={"format": "pt"})
            torch.save(self.optimizer_state_dict(), os.path.join(output_dir, "optimizer.bin"))
            torch.save(self.scheduler_state_dict(), os.path.join(output_dir, "scheduler.bin"))
            if self.scaler is not None:     # accelerator.save_state writes the fp16 GradScaler as scaler.pt
                torch.save(self.scaler.state_dict(), os.path.join(output_dir, "scaler.pt"))
        torch.save({"torch_manual_seed": torch.get_rng_state(), "step": self.step},
                   os.path.join(output_dir, f"random_states_{rank}.pkl"))

    def load_state(self, input_dir):
        """accelerator.load_state(dir) equivalent: student weights, optimizer moments and step.
        Files are read with safe loaders only (safetensors; torch.load(weights_only=True))."""
        self.flush()
        from safetensors.torch import load_file
        sd = load_file(os.path.join(input_dir, "model.safetensors"))
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        self.s.load_state_dict(sd, strict=False)
        self.s.sync_bf16()
        opt = torch.load(os.path.join(input_dir, "optimizer.bin"), map_location="cpu", weights_only=True)
        self.load_optimizer_state_dict(opt)
        cp = os.path.join(input_dir, "scaler.pt")
        if self.scaler is not None and os.path.exists(cp):
            self.scaler.load_state_dict(torch.load(cp, map_location="cpu", weights_only=True))
        sp = os.path.join(input_dir, "scheduler.bin")
        if os.path.exists(sp):
            sch = torch.load(sp, map_location="cpu", weights_only=True)
            if int(sch["last_epoch"]) != self.step * self.world:
                raise ValueError(f"scheduler last_epoch {sch['last_epoch']} != step {self.step} x world {self.world}")
        self.micro = 0
        self.s.grad.zero_()
