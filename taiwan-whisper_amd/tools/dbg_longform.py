"""Debug aid for the long-form timestamp test: window 0 of the 65 s input; at every emitted position
compare (a) the bf16-autocast oracle's rule-processed row, (b) our engine's full-forward
(teacher-forced) row, and print where the emitted token is not the processed argmax of either."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "taiwan-whisper_amd"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch

import make_golden as mg
from oracle import greedy_ref
from oracle.weights import CONFIGS, make_weights
from oracle.whisper_ref import Ref, to_torch
from tw.config import GenerationConfig, WhisperConfig
from tw.modeling import WhisperForConditionalGeneration

cfg = CONFIGS["micro"]
w = make_weights(cfg, 1, lin_std=0.2)
m = WhisperForConditionalGeneration.from_state_dict(WhisperConfig(**cfg), {k: torch.from_numpy(v) for k, v in w.items()},
                                                    dtype=torch.float32)
gc = mg.ts_generation_config().to_dict()
m.generation_config = GenerationConfig(**{k: gc[k] for k in (
    "decoder_start_token_id", "eos_token_id", "pad_token_id", "suppress_tokens", "begin_suppress_tokens", "max_length",
    "no_timestamps_token_id", "is_multilingual", "lang_to_id", "task_to_id", "max_initial_timestamp_index")})
lf = torch.from_numpy(mg.longform_features())
trace = []
m.generate(lf, attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True, language="zh",
           task="transcribe", _trace=trace)
prompt = [50258, 50260, 50359]
ref = Ref(cfg, to_torch(w), amp=True)
sup = mg.SUPPRESS
tr = trace[0]
toks = tr["raw"]
print("window 0: seek", tr["seek"], "tokens", len(toks))
seg = torch.zeros(1, 80, 3000)
seg[0] = lf[0, :, :3000]
seq = torch.tensor([prompt + toks])
with torch.no_grad():
    lg = ref.logits(ref.decoder(seq[:, :-1], ref.encoder(seg))).float()[0]
out = m(input_features=seg.to("cuda"), decoder_input_ids=seq[:, :-1].to("cuda"))
ours = (out["logits"] if isinstance(out, dict) else out.logits).float().cpu()[0]
P = len(prompt)
for j, tok in enumerate(toks):
    if j > 0 and toks[j - 1] == 50257:
        break
    rows = []
    for src in (lg, ours):
        row = src[P - 1 + j, :lg.shape[-1]].clone()
        row[sup] = -float("inf")
        if j == 0:
            row[[220, 50257]] = -float("inf")
        rows.append(greedy_ref.timestamp_rules(row, toks[:j], j == 0, max_initial=50))
    o, u = rows
    raw_d = float((lg[P - 1 + j] - ours[P - 1 + j, :lg.shape[-1]]).abs().max())
    flag = "" if int(o.argmax()) == tok and int(u.argmax()) == tok else "  <--"
    print(f"j={j:3d} tok={tok} oracle argmax={int(o.argmax())} ({float(o.max()):.3f}, tok {float(o[tok]):.3f}) "
          f"ours-fwd argmax={int(u.argmax())} ({float(u.max()):.3f}, tok {float(u[tok]):.3f}) raw max|d|={raw_d:.3f}{flag}")

# the timestamp select kernel on our own full-forward rows at a few positions (state rebuilt from
# the emitted tokens): its pick vs the oracle rules on the same row
from tw import ops
V = lg.shape[-1]
supb = ops.token_bitmask(sup, V, "cuda")
begb = ops.token_bitmask([220, 50257], V, "cuda")
for j in (42, 43, 44, 45, 46):
    row = ours[P - 1 + j, :].to(torch.bfloat16).cuda().contiguous()
    Vp = row.numel()
    ids = torch.tensor([prompt + toks[:j] + [0]], dtype=torch.int64, device="cuda")
    ts_hist = [t for t in toks[:j] if t >= 50364]
    last = torch.tensor([ts_hist[-1] if ts_hist else -1], dtype=torch.int32, device="cuda")
    done = torch.zeros(1, dtype=torch.uint8, device="cuda")
    nxt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ops.greedy_select_ts(row, Vp, 1, V, supb, begb, 50257, done, ids, P + j, nxt, last, P, max_initial=50)
    torch.cuda.synchronize()
    r = ours[P - 1 + j, :V].clone()
    r[sup] = -float("inf")
    pr = greedy_ref.timestamp_rules(r, toks[:j], j == 0, max_initial=50)
    pre = greedy_ref.timestamp_rules(r, toks[:j], j == 0, max_initial=50, apply_mass=False)
    print(f"select j={j}: kernel {int(nxt.item())}  oracle-rules {int(pr.argmax())}  emitted {toks[j]}  "
          f"ts_lse {float(pre[50364:].logsumexp(-1)):.3f} text max {float(pre[:50364].max()):.3f} "
          f"(id {int(pre[:50364].argmax())}) last_ts {int(last.item())}")
