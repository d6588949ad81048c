"""ORACLE — test infrastructure only. NOT part of the product.

CPU restatement of the taiwan-whisper distillation hot path
(`training/run_distillation.py` train_step, `training/create_student_model.py`,
`utils/model_utils.py`) and of the third-party arithmetic it calls
(HF Transformers Whisper forward / feature extractor, torch AdamW / clip).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import anything from here, and only as the checker / CPU baseline — never as the
thing measured or shipped.  The product (`taiwan-whisper_amd/tw`) never imports
this package and fails loudly when its HIP library is missing.

Pinning: every function here is checked against golden vectors produced by the
real reference arithmetic (HF Transformers 5.15 WhisperForConditionalGeneration /
WhisperFeatureExtractor, and the reference's own `create_student_model.py` /
`model_utils.py` imported from /root/reference) by `tests/golden/make_golden.py`;
see `tests/test_oracle_golden.py`.  The `run_distillation.py` closures
(`kl_divergence`, `train_step`, collator) cannot be imported (the script fails on
`import evaluate`), so they are restated from source text and pinned on the HF
model outputs they consume plus hand-derived collator cases.

Modules:
  weights     – documented PRNG weight generator (numpy PCG64) for parity tests
  logmel      – WhisperFeatureExtractor restatement (numpy float64)
  labels      – prepare_train_dataset label logic + DataCollatorSpeechSeq2SeqWithPadding
  whisper_ref – torch-CPU Whisper forward with CUDA-autocast bf16 rounding points
  distill_ref – kl_divergence / train_step / eval_step / AdamW+clip step
  student_ref – init_student_model_from_teacher layer map, mix_language_embeddings
  greedy_ref  – greedy decode restatement (HF generate num_beams=1)
"""
