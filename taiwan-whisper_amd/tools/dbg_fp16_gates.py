"""Debug: per-step log-probs of the fp16 long-form windows (engine device gates vs engine teacher-forced logits vs
the fp16 oracle on CPU).  Dev tool, not product."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "taiwan-whisper_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
from test_fp16_gpu import _model  # noqa: E402
import make_golden as mg  # noqa: E402
from oracle import greedy_ref  # noqa: E402
from oracle.weights import CONFIGS, make_weights  # noqa: E402
from oracle.whisper_ref import Ref, to_torch  # noqa: E402

m, _ = _model(lin_std=0.2, ts=True)
lf = torch.from_numpy(mg.longform_features())
kw = dict(attention_mask=torch.ones(1, lf.shape[-1], dtype=torch.long), return_timestamps=True, language="zh",
          task="transcribe")
trace = []
m.generate(lf, temperature=(0.0,), logprob_threshold=-1e9, no_speech_threshold=1.0, _trace=trace, **kw)
h = np.load(os.path.join(REPO, "tests", "golden", "fp16.npz"))
cfg = CONFIGS["micro"]
ref = Ref(cfg, to_torch(make_weights(cfg, 1, lin_std=0.2), torch.float16), amp=True, stream_bf16=True,
          half=torch.float16)
for i, t in enumerate(trace):
    seg = torch.zeros(1, 80, 3000)
    seg[0, :, :t["n"]] = lf[0, :, t["seek"]:t["seek"] + t["n"]]
    raw, P = list(t["raw"]), len(t["prompt"])
    dec = torch.tensor([t["prompt"] + raw[:-1]])
    lg_e = m(input_features=seg.cuda(), decoder_input_ids=dec.cuda()).logits[0].float().cpu()
    with torch.no_grad():
        lg_o = ref.forward(seg, dec)["logits"][0].float()
    lps = []
    for name, lg in (("engine", lg_e), ("oracle", lg_o)):
        out = []
        for j, tok in enumerate(raw):
            row = lg[P - 1 + j].clone()
            row[mg.SUPPRESS] = -float("inf")
            if j == 0:
                row[[220, 50257]] = -float("inf")
            r = greedy_ref.timestamp_rules(row, raw[:j], j == 0, max_initial=50)
            out.append(float(torch.log_softmax(r, -1)[tok]))
        lps.append(out)
    cand = list(raw)
    while len(cand) > 1 and cand[-1] == 50257 and cand[-2] == 50257:
        cand = cand[:-1]
    n = len(cand)
    print(f"window {i}: seek {t['seek']} n_tok {n} device avg {t['avg_logprob']:.5f} HF {h['f16_fb_avg_logprobs'][i]:.5f} "
          f"engine-TF {sum(lps[0][:n]) / n:.5f} oracle {sum(lps[1][:n]) / n:.5f}")
    for j in range(n):
        d = lps[0][j] - lps[1][j]
        if abs(d) > 0.01:
            print(f"   step {j} tok {raw[j]} engine {lps[0][j]:.4f} oracle {lps[1][j]:.4f} logit diff max "
                  f"{float((lg_e[P - 1 + j] - lg_o[P - 1 + j]).abs().max()):.4f}")
