"""WhisperConfig: the HF `config.json` fields the reference reads
(`training/run_distillation.py:984-1030`, `training/create_student_model.py:131-137`).
Unknown keys are preserved so a round-trip through save_pretrained keeps the file intact."""
from __future__ import annotations

import copy
import json
import os

DEFAULTS = dict(
    vocab_size=51865, num_mel_bins=80, encoder_layers=4, encoder_attention_heads=6, decoder_layers=4,
    decoder_attention_heads=6, decoder_ffn_dim=1536, encoder_ffn_dim=1536, d_model=384,
    max_source_positions=1500, max_target_positions=448, pad_token_id=50257, bos_token_id=50257,
    eos_token_id=50257, decoder_start_token_id=50258, activation_function="gelu", scale_embedding=False,
    dropout=0.0, attention_dropout=0.0, activation_dropout=0.0, layerdrop=0.0, encoder_layerdrop=0.0,
    decoder_layerdrop=0.0, tie_word_embeddings=True, model_type="whisper",
)


class WhisperConfig:
    def __init__(self, **kw):
        d = dict(DEFAULTS)
        d.update(kw)
        self.__dict__.update(d)
        if self.activation_function not in ("gelu",):
            raise NotImplementedError(f"activation {self.activation_function}")
        if self.d_model % self.encoder_attention_heads or self.d_model // self.encoder_attention_heads != 64:
            raise NotImplementedError("tw kernels are specialised for head_dim 64 (every Whisper size)")
        if self.scale_embedding:
            raise NotImplementedError("scale_embedding=True is not used by any Whisper checkpoint")

    @property
    def head_dim(self):
        return self.d_model // self.encoder_attention_heads

    def to_dict(self):
        return copy.deepcopy({k: v for k, v in self.__dict__.items() if not k.startswith("_")})

    def update(self, d: dict):
        self.__dict__.update(d)

    @classmethod
    def from_dict(cls, d):
        return cls(**d)

    @classmethod
    def from_pretrained(cls, path):
        with open(os.path.join(path, "config.json")) as f:
            return cls(**json.load(f))

    def save_pretrained(self, path):
        os.makedirs(path, exist_ok=True)
        d = self.to_dict()
        d.setdefault("architectures", ["WhisperForConditionalGeneration"])
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(d, f, indent=2, sort_keys=True)

    def __repr__(self):
        return f"WhisperConfig(d_model={self.d_model}, enc={self.encoder_layers}, dec={self.decoder_layers})"


def _dims(d, enc, dec, heads, ffn):
    return dict(d_model=d, encoder_layers=enc, decoder_layers=dec, encoder_attention_heads=heads,
                decoder_attention_heads=heads, encoder_ffn_dim=ffn, decoder_ffn_dim=ffn)


# architecture dims of the checkpoints the reference names (openai/whisper-* config.json; distil-32-2 is
# create_student_model.py with --decoder_layers 2 from large-v2)
MODEL_DIMS = {
    "tiny": _dims(384, 4, 4, 6, 1536),
    "base": _dims(512, 6, 6, 8, 2048),
    "small": _dims(768, 12, 12, 12, 3072),
    "medium": _dims(1024, 24, 24, 16, 4096),
    "large-v2": _dims(1280, 32, 32, 20, 5120),
    "distil-32-2": _dims(1280, 32, 2, 20, 5120),
}

# openai/whisper-large-v2 generation_config.json suppress_tokens (the multilingual checkpoints' list)
LARGE_V2_SUPPRESS = [1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93,
                     359, 503, 522, 542, 873, 893, 902, 918, 922, 931, 1350, 1853, 1982, 2460, 2627, 3246,
                     3253, 3268, 3536, 3846, 3961, 4183, 4667, 6585, 6647, 7273, 9061, 9383, 10428, 10929,
                     11938, 12033, 12331, 12562, 13793, 14157, 14635, 15265, 15618, 16553, 16604, 18362,
                     18956, 20075, 21675, 22520, 26130, 26161, 26435, 28279, 29464, 31650, 32302, 32470,
                     36865, 42863, 47425, 49870, 50254, 50258, 50358, 50359, 50360, 50361, 50362]


GEN_DEFAULTS = dict(
    decoder_start_token_id=50258, eos_token_id=50257, pad_token_id=50257, bos_token_id=50257,
    no_timestamps_token_id=50363, max_length=448, num_beams=1, suppress_tokens=[], begin_suppress_tokens=[220, 50257],
    is_multilingual=True, lang_to_id={}, task_to_id={"transcribe": 50359, "translate": 50358},
)


class GenerationConfig(dict):
    """`generation_config.json` as a dict (round-trips unchanged) with HF-style attribute access and
    the Whisper defaults for keys the file lacks (HF generation_whisper.py reads these fields)."""

    def __getattr__(self, name):
        if name in self:
            return self[name]
        if name in GEN_DEFAULTS:
            return copy.deepcopy(GEN_DEFAULTS[name])
        raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value

    def to_dict(self):
        return copy.deepcopy(dict(self))
