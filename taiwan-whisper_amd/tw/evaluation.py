"""Evaluation metrics of the distillation loop, host side.

  MixErrorRate            utils/evaluation.py:38-237   (mixed Chinese-character / English-word error rate:
                                                        the string is cut into CJK characters and
                                                        alphanumeric words, punctuation and spaces dropped,
                                                        traditional -> simplified Chinese first)
  cal_single_complete_mer utils/evaluation.py:25-36    (substitution / deletion / insertion counts)
  compute_metrics         training/run_distillation.py:1366-1387 (orthographic and normalised MER x 100
                                                        over decoded predictions / labels)

Third-party pieces the reference imports, restated or gated:
  * editdistance.eval (Levenshtein distance over token lists, unit costs) -> `levenshtein`, an exact
    restatement (row-vectorised DP: d[i][j] = j + cummin_k(t[k] - k) for the insertion chain);
  * edit_distance.SequenceMatcher opcodes -> `_opcodes`, a Levenshtein backtrace; S + D + I equals the
    distance, but how a tie between alignments is broken (and so the split among S, D and I) may
    differ from that package: parity unpinned for the split, pinned for the total;
  * opencc t2s (traditional -> simplified) is not installed in this image: the converter is opencc's
    when importable, else a caller-supplied callable, else none (MER then compares characters as
    written; parity for mixed-script inputs unpinned);
  * pypinyin / the lexicon file of `phonemize=True` are absent: that mode raises.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, List, Optional, Sequence

import numpy as np

_SEPARATORS = frozenset([' ', '\t', '\n', '\r', ',', '.', '!', '?', '。', '，', '！', '？', '、', '；', '：', '「', '」', '『',
                         '』', '（', '）', '(', ')', '\\[', '\\]', '{', '}', '<', '>', '《', '》', '“', '”', '‘', '’', '…', '—',
                         '～', '·', '•'])   # '\\[' and '\\]' are 2-char strings in the reference: never match


def levenshtein(a: Sequence, b: Sequence) -> int:
    """Unit-cost edit distance between two sequences of hashable items (editdistance.eval)."""
    if len(a) == 0:
        return len(b)
    if len(b) == 0:
        return len(a)
    vocab: dict = {}
    ia = np.array([vocab.setdefault(x, len(vocab)) for x in a], dtype=np.int64)
    ib = np.array([vocab.setdefault(x, len(vocab)) for x in b], dtype=np.int64)
    n = len(ib)
    ar = np.arange(n + 1, dtype=np.int64)
    prev = ar.copy()
    for i in range(1, len(ia) + 1):
        t = np.empty(n + 1, dtype=np.int64)
        t[0] = i
        t[1:] = np.minimum(prev[1:] + 1, prev[:-1] + (ib != ia[i - 1]))
        prev = ar + np.minimum.accumulate(t - ar)
    return int(prev[-1])


def _opcodes(ref: Sequence, hyp: Sequence):
    """Levenshtein alignment as (tag, i1, i2, j1, j2) runs (tags: equal / replace / delete / insert)."""
    n, m = len(ref), len(hyp)
    d = np.zeros((n + 1, m + 1), dtype=np.int64)
    d[:, 0] = np.arange(n + 1)
    d[0, :] = np.arange(m + 1)
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            d[i, j] = min(d[i - 1, j] + 1, d[i, j - 1] + 1, d[i - 1, j - 1] + (ref[i - 1] != hyp[j - 1]))
    ops = []
    i, j = n, m
    while i > 0 or j > 0:
        if i > 0 and j > 0 and d[i, j] == d[i - 1, j - 1] + (ref[i - 1] != hyp[j - 1]):
            ops.append(("equal" if ref[i - 1] == hyp[j - 1] else "replace", i - 1, i, j - 1, j))
            i, j = i - 1, j - 1
        elif i > 0 and d[i, j] == d[i - 1, j] + 1:
            ops.append(("delete", i - 1, i, j, j))
            i -= 1
        else:
            ops.append(("insert", i, i, j - 1, j))
            j -= 1
    return ops[::-1]


def cal_single_complete_mer(ref, hyp):
    ops = _opcodes(ref, hyp)
    s = sum(max(x[2] - x[1], x[4] - x[3]) for x in ops if x[0] == "replace")
    d = sum(max(x[2] - x[1], x[4] - x[3]) for x in ops if x[0] == "delete")
    i = sum(max(x[2] - x[1], x[4] - x[3]) for x in ops if x[0] == "insert")
    return s, d, i, len(ref)


def cal_complete_mer(ref_data, hyp_data):
    S = D = I = N = count = 0
    for ref, hyp in zip(ref_data, hyp_data):
        _s, _d, _i, _n = cal_single_complete_mer(ref, hyp)
        S, D, I, N, count = S + _s, D + _d, I + _i, N + _n, count + 1
    return S, D, I, N, count


def _is_cjk(ch: str) -> bool:
    return u'一' <= ch <= u'鿿'


class MixErrorRate:
    def __init__(self, to_simplified_chinese=True, to_traditional_chinese=False, phonemize=False,
                 separate_language=False, test_only=False, count_repetitive_hallucination=False,
                 calculate_complete_mer=False, converter: Optional[Callable[[str], str]] = None):
        if to_simplified_chinese and to_traditional_chinese:
            raise ValueError("Can't convert to both simplified and traditional chinese at the same time.")
        if phonemize:
            raise NotImplementedError("phonemize=True needs pypinyin and the reference's lexicon file "
                                      "(utils/evaluation.py:68-84), neither of which is available here")
        self.converter = converter
        if self.converter is None and (to_simplified_chinese or to_traditional_chinese):
            try:
                import opencc  # the reference's converter (absent in this image)
                cc = opencc.OpenCC("t2s.json" if to_simplified_chinese else "s2t.json")
                self.converter = cc.convert
            except ImportError:
                self.converter = None
        self.phonemize = phonemize
        self.test_only = test_only
        self.separate_language = separate_language
        self.count_repetitive_hallucination = count_repetitive_hallucination
        self.calculate_complete_mer = calculate_complete_mer

    def _from_str_to_list(self, cs_string: str) -> List[str]:
        out, word = [], ''
        for s in cs_string:
            if s in _SEPARATORS:
                if word:
                    out.append(word)
                    word = ''
                continue
            if _is_cjk(s):
                if word:
                    out.append(word)
                    word = ''
                out.append(self.converter(s) if self.converter is not None else s)
            elif s.isalnum() or s in ("'", "-"):
                word += s
            # else: an unknown character, dropped (the reference prints it)
        if word:
            out.append(word)
        return out

    @staticmethod
    def _unit_is_en(token):
        return not _is_cjk(token[0])

    @staticmethod
    def _unit_is_zh(token):
        return _is_cjk(token[0])

    @staticmethod
    def _count_repetitive_hallucination(cs_str, n=6, repeat=5, reset_len=100):
        count = 0
        counts = defaultdict(int)
        if len(cs_str) < n:
            return 0
        prev_reset = 0
        for i in range(len(cs_str) - n + 1):
            g = cs_str[i:i + n]
            if '|>' in g or '<|' in g:
                continue
            counts[g] += 1
            if counts[g] >= repeat:
                count += 1
                counts = defaultdict(int)
            if i - prev_reset >= reset_len:
                counts = defaultdict(int)
                prev_reset = i
        return count

    def compute(self, predictions=None, references=None, show_progress=False, empty_error_rate=1.0, **kw):
        total_err = total_ref = en_err = en_ref = zh_err = zh_ref = 0
        rep_h = rep_r = 0
        if self.test_only:
            predictions, references = predictions[:10], references[:10]
        S = D = I = N = 0
        for pred, ref in zip(predictions, references):
            if self.count_repetitive_hallucination:
                rep_h += self._count_repetitive_hallucination(pred)
                rep_r += self._count_repetitive_hallucination(ref)
            pl, rl = self._from_str_to_list(pred), self._from_str_to_list(ref)
            if self.calculate_complete_mer:
                _s, _d, _i, _n = cal_single_complete_mer(rl, pl)
                S, D, I, N = S + _s, D + _d, I + _i, N + _n
            if self.separate_language:
                ep, er = [t for t in pl if self._unit_is_en(t)], [t for t in rl if self._unit_is_en(t)]
                zp, zr = [t for t in pl if self._unit_is_zh(t)], [t for t in rl if self._unit_is_zh(t)]
                en_err += levenshtein(ep, er)
                en_ref += len(er)
                zh_err += levenshtein(zp, zr)
                zh_ref += len(zr)
            total_err += levenshtein(pl, rl)
            total_ref += len(rl)
        if total_ref == 0:
            return empty_error_rate
        mer = total_err / total_ref
        if self.separate_language or self.count_repetitive_hallucination:
            res = {"MER": mer}
            if self.separate_language:
                res["EN WER"] = en_err / en_ref if en_ref else 0
                res["ZH CER"] = zh_err / zh_ref if zh_ref else 0
            if self.count_repetitive_hallucination:
                res["Hyp Repetitive Hallucination Count"] = rep_h
                res["Ref Repetitive Hallucination Count"] = rep_r
            return res
        return mer


def default_normalizer(language: Optional[str] = "zh", english_spelling_normalizer: Optional[dict] = None):
    """run_distillation.py:1144-1148: BasicTextNormalizer when a language is set, else the English one."""
    from transformers.models.whisper.english_normalizer import BasicTextNormalizer, EnglishTextNormalizer
    if language is not None:
        return BasicTextNormalizer()
    return EnglishTextNormalizer(english_spelling_normalizer or {})


def compute_metrics(preds, labels, tokenizer, metric: Optional[MixErrorRate] = None, normalizer=None,
                    return_timestamps: bool = False):
    """run_distillation.py:1366-1387 -> ({"wer", "wer_ortho"}, pred_str, label_str, norm_pred, norm_label)."""
    metric = metric or MixErrorRate()
    normalizer = normalizer or default_normalizer()
    labels = [np.where(np.asarray(l) == -100, tokenizer.pad_token_id, np.asarray(l)) for l in labels]
    preds = [np.asarray(p) for p in preds]
    try:
        pred_str = tokenizer.batch_decode(preds, skip_special_tokens=True, decode_with_timestamps=return_timestamps)
    except TypeError:
        pred_str = tokenizer.batch_decode(preds, skip_special_tokens=True)
    label_str = tokenizer.batch_decode(labels, skip_special_tokens=True)
    wer_ortho = 100 * metric.compute(predictions=pred_str, references=label_str)
    norm_pred = [normalizer(p) for p in pred_str]
    norm_label = [normalizer(l) for l in label_str]
    keep = [i for i in range(len(norm_label)) if len(norm_label[i]) > 0]
    pred_str = [pred_str[i] for i in keep]
    label_str = [label_str[i] for i in keep]
    norm_pred = [norm_pred[i] for i in keep]
    norm_label = [norm_label[i] for i in keep]
    wer = 100 * metric.compute(predictions=norm_pred, references=norm_label)
    return {"wer": wer, "wer_ortho": wer_ortho}, pred_str, label_str, norm_pred, norm_label
