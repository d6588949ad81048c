"""Diagnostics for tests/test_lv2_decode_gpu.py failures: the fp32 long-form's first differing token against HF's
margin there, and the fp16 / bf16 teacher-forced step logits (engine top-2, HF token's logit) at the first
disagreement.  python tools/dbg_lv2.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np
import torch


def main():
    import threading
    import time

    def beat():
        while True:
            time.sleep(50)
            print("[dbg] alive", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    import test_lv2_decode_gpu as T
    mg = T._mg()
    from oracle.weights import lv2_decode_weights, CONFIGS
    g = T.load_golden("lv2_decode")
    w = {k: torch.from_numpy(v) for k, v in lv2_decode_weights(CONFIGS["large-v2"], int(g["seed"])).items()}
    lv2 = (mg, g, w)
    short, lf = mg.lv2_features()
    for arith, dt, tag in (() if "--long-only" in sys.argv else (("fp16", torch.float16, "f16"), ("bf16", torch.float32, "b16"))):
        m = T._model(lv2, dt, arith, ts=False)      # bf16: fp32 parameters under autocast, as HF's fixture
        want = g[f"{tag}_greedy_ids"]
        margin = g[f"{tag}_greedy_margin"].T
        from tw.generation import DecodeSession
        dev = m.device
        enc16 = m.encode(m.conv_input(torch.from_numpy(short).to(dev, torch.float32)))
        print(arith, "enc finite", bool(torch.isfinite(enc16.float()).all()), "enc absmax", float(enc16.float().abs().max()))
        B, S = want.shape
        prompt = g["prompt"].tolist()
        sess = DecodeSession(m, enc16, B, enc16.shape[0] // B, len(prompt) + S + 1)
        sess.t_dev.zero_()
        for t in prompt[:-1]:
            sess.cur.fill_(int(t))
            sess.step()
        sess.cur.fill_(int(prompt[-1]))
        V = m.config.vocab_size
        sup = torch.tensor(mg.SUPPRESS, device=dev)
        fd = torch.from_numpy(np.ascontiguousarray(want)).to(dev, torch.int64)
        shown = 0
        agree = total = 0
        mism = []
        for t in range(S):
            sess.step()
            lg = sess.logits[:, :V].float()
            lg[:, sup] = -float("inf")
            if t == 0:
                lg[:, [220, 50257]] = -float("inf")
            top = lg.topk(2, -1)
            for r in range(B):
                total += 1
                if int(top.indices[r, 0]) == int(want[r, t]):
                    agree += 1
                else:
                    mism.append((float(margin[r, t]), float(top.values[r, 0])))
                if int(top.indices[r, 0]) != int(want[r, t]) and shown < 6:
                    shown += 1
                    print(f"{arith} row {r} step {t}: engine top2 {top.indices[r].tolist()} {top.values[r].tolist()} "
                          f"HF token {int(want[r, t])} engine logit there {float(lg[r, int(want[r, t])]):.4f} "
                          f"HF margin {float(margin[r, t]):.4f}  x absmax {float(sess.x.float().abs().max()):.1f} "
                          f"finite {bool(torch.isfinite(sess.logits.float()).all())}", flush=True)
            sess.cur.copy_(fd[:, t])
        print(f"{arith}: teacher-forced agreement {agree}/{total}; mismatch HF margins (sorted) "
              f"{sorted(round(a, 3) for a, _ in mism)}; top logits {[round(b, 1) for _, b in mism][:8]}", flush=True)
        del m, sess
        torch.cuda.empty_cache()
    # fp32 long-form
    m = T._model(lv2, torch.float32, "fp32", ts=True)
    lt = torch.from_numpy(lf)
    trace = []
    long = m.generate(lt, attention_mask=torch.ones(1, lt.shape[-1], dtype=torch.long), return_timestamps=True,
                      language="zh", task="transcribe", temperature=(0.0,), logprob_threshold=-1e9,
                      no_speech_threshold=1.0, _trace=trace).cpu().numpy()[0]
    want = g["f32_long_ids"][0]
    n = min(len(long), len(want))
    diff = np.nonzero(long[:n] != want[:n])[0]
    print("fp32 long: lens", len(long), len(want), "first diff", diff[:3].tolist())
    steps = g["f32_long_window_steps"].tolist()
    lm = g["f32_long_margin"]
    print("engine windows", [(t["seek"], len(t["raw"])) for t in trace])
    print("HF window steps", steps, "HF avg", g["f32_long_avg_logprobs"].tolist())
    print("engine avg", [round(t["avg_logprob"], 6) for t in trace])
    # first differing raw token per window vs HF's window raw (not stored): report the HF margins' smallest values
    # engine output per window (segments concatenated in order) -> window of the first difference
    if len(diff):
        i0, acc = int(diff[0]), 0
        for wi, t in enumerate(trace):
            nseg = len(t["raw"])
            print(f"  window {wi} seek {t['seek']} raw {nseg}")
        print("  first diff at output index", i0, "engine", long[i0 - 2:i0 + 3].tolist(), "HF", want[i0 - 2:i0 + 3].tolist())
    print("HF long margins: min", float(lm.min()), "count < 1e-4", int((lm < 1e-4).sum()), "< 1e-3", int((lm < 1e-3).sum()),
          "positions < 1e-3", np.nonzero(lm < 1e-3)[0][:10].tolist())


if __name__ == "__main__":
    main()
