"""Size-independent properties of the distillation step at BASELINE config 3's full size (VERDICT r01
item 2): distil-32-2 student made by the create_student_model layer map from a random-init large-v2
teacher, frozen shared encoder, B = 64 synthetic 30 s clips (GPU log-mel) -- the bench workload, where
the CPU oracle cannot follow (its parity is pinned at the same dims with B = 1 in test_configs_gpu.py).

  * the loss, CE and KL are finite and the gradient norm is finite and non-zero;
  * the loss is the token-weighted combination of the two half-batches' losses (the reference's
    per-batch normalisation, run_distillation.py:1539-1551: CE mean over valid tokens + KL sum / valid
    tokens), 1e-3 relative -- the halves run different GEMM tilings (M = 28608 vs 14304);
  * the step is deterministic: two runs from the same weights give bit-identical losses and parameters
    (no atomics on the path; every reduction has a fixed order).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_c3_full_size_properties():
    from tw.config import MODEL_DIMS, WhisperConfig
    from tw.data import DataCollatorSpeechSeq2SeqWithPadding, synthetic_audio, synthetic_label_lists
    from tw.distill import DistillationTrainer
    from tw.feature_extraction import WhisperFeatureExtractor
    from tw.modeling import WhisperForConditionalGeneration, random_init_
    from tw.student import student_from_teacher
    B = 64
    tcfg = WhisperConfig(**MODEL_DIMS["large-v2"])
    t32 = random_init_(WhisperForConditionalGeneration(tcfg, dtype=torch.float32, device=DEV), seed=0)
    student, _, _ = student_from_teacher(t32, encoder_layers=32, decoder_layers=2)
    teacher = WhisperForConditionalGeneration(tcfg, dtype=torch.bfloat16, device=DEV)
    teacher.store.p16.copy_(t32.store.p16)
    teacher._refresh_ln32()
    del t32
    torch.cuda.empty_cache()
    fe = WhisperFeatureExtractor(device=DEV)
    _, conv = fe.extract(synthetic_audio(B, seed=5, device=DEV))
    dec, lab = DataCollatorSpeechSeq2SeqWithPadding(max_target_length=448).collate_labels(
        synthetic_label_lists(B, seed=5))
    dec, lab = dec.to(DEV), lab.to(DEV)
    p0 = student.store.p32.clone()

    def fresh():
        student.store.p32.copy_(p0)
        student.sync_bf16()
        return DistillationTrainer(student, teacher, learning_rate=1e-4, warmup_steps=0, freeze_encoder=True)

    # token-weighted halves (eval_step: no update, the same loss normalisation)
    tr = fresh()
    full = {k: float(v) for k, v in tr.eval_step(dict(conv_input=conv, decoder_input_ids=dec, labels=lab)).items()}
    halves = []
    for sl in (slice(0, B // 2), slice(B // 2, B)):
        m = tr.eval_step(dict(conv_input=conv[sl].contiguous(), decoder_input_ids=dec[sl].contiguous(),
                              labels=lab[sl].contiguous()))
        halves.append(({k: float(v) for k, v in m.items()}, int((lab[sl] != -100).sum())))
    n = sum(c for _, c in halves)
    for k in ("loss", "ce_loss", "kl_loss"):
        comb = sum(h[k] * c for h, c in halves) / n
        print(f"c3 B=64 {k}: full {full[k]:.6f}, token-weighted halves {comb:.6f}")
        assert abs(full[k] - comb) <= 1e-3 * abs(full[k]), k
    # two training steps from the same state: finite and bit-identical
    runs = []
    for _ in range(2):
        tr = fresh()
        m = tr.train_step(dict(conv_input=conv, decoder_input_ids=dec, labels=lab))
        torch.cuda.synchronize()
        runs.append(({k: v.clone() for k, v in m.items()}, float(tr.norm), student.store.p32.clone()))
    (m1, g1, w1), (m2, g2, w2) = runs
    for k in ("loss", "ce_loss", "kl_loss"):
        assert torch.isfinite(m1[k]).all(), k
        assert torch.equal(m1[k], m2[k]), k
    assert g1 == g2 and g1 > 0 and g1 == g1 and g1 != float("inf")
    assert torch.equal(w1, w2)
    assert not torch.equal(w1, p0)                  # the update happened
