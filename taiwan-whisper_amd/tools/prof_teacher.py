"""Teacher forward only (large-v2 bf16, encoder + decoder over T_dec 447 + tied head), B clips, for a
per-kernel trace:  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pt -o run -- \
    python3 tools/prof_teacher.py [--batch 64] [--reps 3]
then tools/trace_by_grid.py gpurun_out/pt --reps 3."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from tw.config import MODEL_DIMS, WhisperConfig
    from tw.data import DataCollatorSpeechSeq2SeqWithPadding, synthetic_audio, synthetic_label_lists
    from tw.feature_extraction import WhisperFeatureExtractor
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    dev = torch.device("cuda", 0)
    t = random_init_(WhisperForConditionalGeneration(WhisperConfig(**MODEL_DIMS["large-v2"]), dtype=torch.bfloat16,
                                                     device=dev), seed=0)
    fe = WhisperFeatureExtractor(device=dev)
    _, conv = fe.extract(synthetic_audio(a.batch, seed=0, device=dev))
    dec, _ = DataCollatorSpeechSeq2SeqWithPadding(max_target_length=448).collate_labels(
        synthetic_label_lists(a.batch, seed=0))
    dec = dec.to(dev)
    with torch.no_grad():
        for r in range(a.reps + 1):
            if r == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            enc = t.encode(conv)
            t.lm_head(t.decode(dec, enc, enc.shape[0] // a.batch))
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.reps / a.batch * 1e3
    print(f"teacher fwd {ms:.3f} ms/clip (B={a.batch}, T_dec={dec.shape[1]})", flush=True)


if __name__ == "__main__":
    main()
