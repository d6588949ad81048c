"""ORACLE (test infrastructure only): restatement of the Whisper log-mel front end.

Reference call site: `training/run_distillation.py:1215-1219`
(`feature_extractor(audio, sampling_rate=...)`) which runs
HF:models/whisper/feature_extraction_whisper.py:193-349 (`__call__`: pad/truncate
to 480 000 samples with 0.0) and, because torch is importable, `:135-170`
(`_torch_extract_fbank_features`: torch.stft n_fft 400, hop 160, periodic Hann,
center reflect pad; |.|^2; drop last frame; mel (slaney) matmul; log10(clamp
1e-10); max(x, clip_max - 8) per clip; (x + 4) / 4).

The mel filter bank restates HF:audio_utils.py `mel_filter_bank(201, 80, 0, 8000,
16000, norm="slaney", mel_scale="slaney")`.  Computed here in float64.
"""
from __future__ import annotations

import numpy as np

SR, N_FFT, HOP, N_MELS, N_SAMPLES, N_FRAMES = 16000, 400, 160, 80, 480000, 3000


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    mels = 3.0 * f / 200.0
    min_log_hz, min_log_mel, logstep = 1000.0, 15.0, 27.0 / np.log(6.4)
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) * logstep, mels)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f = 200.0 * m / 3.0
    min_log_hz, min_log_mel, logstep = 1000.0, 15.0, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f)


def mel_filter_bank(n_freqs: int = 201, n_mels: int = N_MELS, fmin: float = 0.0,
                    fmax: float = 8000.0, sr: int = SR) -> np.ndarray:
    """[n_freqs, n_mels] slaney-normalised triangular filters (HF audio_utils)."""
    mel_freqs = np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2)
    filter_freqs = _mel_to_hz(mel_freqs)
    fft_freqs = np.linspace(0, sr // 2, n_freqs)
    diff = np.diff(filter_freqs)
    slopes = filter_freqs[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    enorm = 2.0 / (filter_freqs[2:n_mels + 2] - filter_freqs[:n_mels])
    return fb * enorm[None, :]


def pad_or_trim(wav: np.ndarray, n: int = N_SAMPLES) -> np.ndarray:
    """HF `__call__` padding='max_length', truncation=True, padding_value 0.0."""
    wav = np.asarray(wav, dtype=np.float64).reshape(-1)[:n]
    out = np.zeros(n, dtype=np.float64)
    out[: wav.shape[0]] = wav
    return out


def log_mel(wav: np.ndarray, n: int = N_SAMPLES) -> np.ndarray:
    """One clip padded / trimmed to n samples -> [80, n // 160] float64 (then compared against float32
    outputs).  n = 480 000 is the 30 s call; the long-form call (HF __call__(truncation=False,
    padding="longest"), run_eval.py:572-581) passes n = the batch's longest clip."""
    x = pad_or_trim(wav, n)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_frames = 1 + (xp.shape[0] - N_FFT) // HOP          # 3001 for 30 s
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(N_FFT) / N_FFT)   # periodic Hann
    spec = np.fft.rfft(xp[idx] * win[None, :], axis=1)     # [3001, 201]
    power = (spec.real ** 2 + spec.imag ** 2)[:-1]          # drop last frame -> [n // 160, 201]
    mel = power @ mel_filter_bank()                         # [3000, 80]
    log_spec = np.log10(np.maximum(mel, 1e-10)).T           # [80, 3000]
    log_spec = np.maximum(log_spec, log_spec.max() - 8.0)
    return (log_spec + 4.0) / 4.0


def log_mel_batch(wavs) -> np.ndarray:
    return np.stack([log_mel(w) for w in wavs]).astype(np.float32)


def log_mel_longest(wavs):
    """HF __call__(truncation=False, padding="longest", return_attention_mask=True): every clip zero-padded
    to the longest one -> (features [B, 80, n // 160] float32, attention mask [B, n // 160] int: one
    entry per hop of real samples, the sample mask rescaled by [::160] and trimmed to the frame count)."""
    n = max(len(w) for w in wavs)
    feats = np.stack([log_mel(w, n) for w in wavs]).astype(np.float32)
    nfr = n // HOP
    mask = np.zeros((len(wavs), nfr), dtype=np.int64)
    for i, w in enumerate(wavs):
        sm = np.zeros(n, dtype=np.int64)
        sm[:len(w)] = 1
        mask[i] = sm[::HOP][:nfr]
    return feats, mask


def synthetic_clip(i: int, seconds: float = 30.0) -> np.ndarray:
    """x_i(t) = 0.5 sin(2π(220+37 i) t) + 0.01 N(0,1), PCG64 seed 1234+i."""
    n = int(seconds * SR)
    t = np.arange(n, dtype=np.float64) / SR
    rng = np.random.Generator(np.random.PCG64(1234 + i))
    return (0.5 * np.sin(2 * np.pi * (220 + 37 * i) * t) + 0.01 * rng.standard_normal(n)).astype(np.float32)
