"""WhisperFeatureExtractor drop-in with the log-mel computed on the GPU.

Reference: `training/run_distillation.py:1215-1219` calls
`feature_extractor(audio, sampling_rate=16000).input_features`; `DataCollatorSpeechSeq2SeqWithPadding`
calls `feature_extractor.pad({"input_features": ...}, padding="longest", return_tensors="pt")`
(`:471-481`).  Arithmetic as HF feature_extraction_whisper.py:135-170 (see csrc/logmel.hip).

The constant tables (DFT basis with the periodic Hann window folded in, and the sparse
slaney mel filter bank of HF audio_utils.mel_filter_bank(201, 80, 0, 8000, 16000,
norm="slaney", mel_scale="slaney")) are built once on the host in float64.
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from . import ops

SAMPLING_RATE, N_FFT, HOP, N_MELS, N_SAMPLES, N_FRAMES = 16000, 400, 160, 80, 480000, 3000
MELW = 32


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * (27.0 / np.log(6.4)), 3.0 * f / 200.0)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= 15.0, 1000.0 * np.exp((np.log(6.4) / 27.0) * (m - 15.0)), 200.0 * m / 3.0)


def mel_filters(n_freqs=201, n_mels=N_MELS, fmin=0.0, fmax=8000.0, sr=SAMPLING_RATE) -> np.ndarray:
    """[n_freqs, n_mels] float64 slaney filter bank."""
    ff = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fft_freqs = np.linspace(0, sr // 2, n_freqs)
    diff = np.diff(ff)
    slopes = ff[None, :] - fft_freqs[:, None]
    fb = np.maximum(0.0, np.minimum(-slopes[:, :-2] / diff[:-1], slopes[:, 2:] / diff[1:]))
    return fb * (2.0 / (ff[2:n_mels + 2] - ff[:n_mels]))[None, :]


@functools.lru_cache(maxsize=None)
def _host_tables():
    n = np.arange(N_FFT, dtype=np.float64)
    win = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / N_FFT)             # periodic Hann
    k = np.arange(201, dtype=np.float64)
    ang = 2.0 * np.pi * np.outer(n, k) / N_FFT
    basis = np.zeros((N_FFT, 416), dtype=np.float64)
    basis[:, :201] = win[:, None] * np.cos(ang)
    basis[:, 208:208 + 201] = -win[:, None] * np.sin(ang)
    fb = mel_filters()                                             # [201, 80]
    start = np.zeros(N_MELS, dtype=np.int32)
    w = np.zeros((N_MELS, MELW), dtype=np.float32)
    for m in range(N_MELS):
        nz = np.nonzero(fb[:, m])[0]
        if nz.size == 0:
            continue
        s, e = int(nz[0]), int(nz[-1]) + 1
        if e - s > MELW:
            raise RuntimeError("mel filter wider than the kernel's tap budget")
        start[m] = s
        w[m, : e - s] = fb[s:e, m].astype(np.float32)
    return basis.astype(np.float32), start, w


def mel_tables(device="cpu"):
    b, s, w = _host_tables()
    return torch.from_numpy(b).to(device), torch.from_numpy(s).to(device), torch.from_numpy(w).to(device)


class WhisperFeatureExtractor:
    """Drop-in for the two calls the reference makes.  `__call__` returns an object with
    `.input_features` ([B, 80, 3000] fp32 on `device`); the time-major bf16 conv1 input is
    also produced (`.conv_input`) so the encoder can skip a transpose."""

    model_input_names = ["input_features"]

    def __init__(self, feature_size=80, sampling_rate=SAMPLING_RATE, hop_length=HOP, chunk_length=30, n_fft=N_FFT,
                 padding_value=0.0, device="cuda"):
        if (feature_size, sampling_rate, hop_length, chunk_length, n_fft) != (80, 16000, 160, 30, 400):
            raise NotImplementedError("tw log-mel kernel is specialised for Whisper's 80x3000 front end")
        self.feature_size, self.sampling_rate, self.padding_value = feature_size, sampling_rate, padding_value
        self.n_samples, self.nb_max_frames = N_SAMPLES, N_FRAMES
        self.device = device
        self._tables = None

    def _tabs(self):
        if self._tables is None:
            self._tables = mel_tables(self.device)
        return self._tables

    @property
    def mel_filters(self):
        return mel_filters().astype(np.float32)

    @staticmethod
    def _as_list(raw_speech):
        if isinstance(raw_speech, (np.ndarray, torch.Tensor)) and getattr(raw_speech, "ndim", 1) == 1:
            return [raw_speech]
        return list(raw_speech)

    def pad_waveforms(self, raw_speech, n: int = N_SAMPLES) -> torch.Tensor:
        """Zero-pad / truncate every clip to n samples (HF __call__: padding='max_length' to 480 000 with
        truncation=True by default; n = the longest clip for padding='longest', truncation=False)."""
        raw_speech = self._as_list(raw_speech)
        out = torch.zeros(len(raw_speech), n, dtype=torch.float32)
        for i, w in enumerate(raw_speech):
            w = torch.as_tensor(np.asarray(w, dtype=np.float32)).reshape(-1)[:n]
            out[i, : w.shape[0]] = w
        return out

    def extract(self, wav: torch.Tensor, want_conv_input: bool = True):
        """wav: [B, n] fp32 (host or device) -> (mel [B,80,n//160] fp32, conv_in [B,n//160+2,80] bf16);
        n = 480 000 for 30 s clips, any n > 200 for long-form inputs."""
        wav = wav.to(self.device, torch.float32).contiguous()
        B, n = wav.shape
        nfr = n // HOP
        basis, start, w = self._tabs()
        mel = torch.empty(B, N_MELS, nfr, dtype=torch.float32, device=self.device)
        conv = torch.empty(B, nfr + 2, N_MELS, dtype=torch.bfloat16, device=self.device) if want_conv_input else None
        ops.logmel(wav, basis, start, w, mel, conv)
        return mel, conv

    def __call__(self, raw_speech, sampling_rate=None, return_tensors=None, truncation=True, padding="max_length",
                 return_attention_mask=None, **kw):
        """HF WhisperFeatureExtractor.__call__ for the reference's two calls: the training default
        (padding='max_length', truncation=True -> [B, 80, 3000]; run_distillation.py:1217) and the long-form
        eval call (truncation=False, padding='longest', return_attention_mask=True -> [B, 80, n_max // 160]
        plus a per-frame mask, run_eval.py:572-581)."""
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(f"expected sampling_rate {self.sampling_rate}, got {sampling_rate}")
        clips = self._as_list(raw_speech)
        lens = [int(np.asarray(c).reshape(-1).shape[0]) for c in clips]
        if padding == "longest":
            n = max(lens) if not truncation else min(max(lens), N_SAMPLES)
        elif padding in ("max_length", True, None):
            n = N_SAMPLES if (truncation or max(lens) <= N_SAMPLES) else max(lens)
        else:
            raise NotImplementedError(f"padding={padding!r}")
        mel, conv = self.extract(self.pad_waveforms(clips, n))
        out = _Features(mel, conv)
        if return_attention_mask:
            nfr = n // HOP
            frame = torch.arange(nfr) * HOP         # the sample mask rescaled by [::hop], trimmed to the frames
            out["attention_mask"] = (frame[None, :] < torch.tensor(lens)[:, None]).to(torch.int32).to(self.device)
        return out

    def pad(self, features: dict, padding="longest", return_tensors="pt", **kw):
        feats = features["input_features"]
        if isinstance(feats, torch.Tensor):
            return {"input_features": feats}
        return {"input_features": torch.stack([torch.as_tensor(f) for f in feats])}


class _Features(dict):
    def __init__(self, mel, conv):
        super().__init__(input_features=mel)
        self.conv_input = conv

    @property
    def input_features(self):
        return self["input_features"]
