"""Host logic of long-form decoding (tw/generation.py _longform) with a scripted stand-in for the device decoder:
the speculative fallback batch must give what decoding the attempts one at a time gives (HF
generate_with_fallback decodes them one by one: generation_whisper.py:970-1090), also when the accepted row of a
batch finishes before another row of that batch on a window that is not the last one."""
import types

import pytest
import torch

from tw import generation
from tw.config import GenerationConfig

EOS = 50257
TS0 = 50364            # <|0.00|>


class _Sel:
    def __init__(self, nb):
        self.sum_logp = torch.zeros(nb)


class _ScriptedDecoder:
    """Stands in for generation._Decoder: row r of a run decodes SCRIPT[(window, temperature)], and the batch is
    cut where its longest row emits eos, the rows that finished earlier padded with eos -- what the device
    decoder returns (DecodeSession ids are eos-filled, _Decoder.run trims at the last row's first eos)."""
    script = {}

    def __init__(self, model, gc, nb, Tk, P, ml, timestamps, use_graph, track=False):
        self.nb = nb
        self.sel = _Sel(nb)
        self.ns_logp = torch.zeros(nb)

    def run(self, enc16, prompt, temperature=0.0, seed=0, no_speech=None):
        # one encoder row per window here: nb rows (one per decode row), or one row shared by every decode row
        ids = enc16.flatten()
        wins = [int(ids[r].item()) if ids.numel() == self.nb else int(ids[0].item()) for r in range(self.nb)]
        temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature]
        assert len(temps) == self.nb
        rows = [list(self.script[(w, round(t, 1))]) for w, t in zip(wins, temps)]
        L = max(len(r) for r in rows)
        for i, r in enumerate(rows):
            self.sel.sum_logp[i] = -0.1 * len(r)
        return torch.tensor([r + [EOS] * (L - len(r)) for r in rows], dtype=torch.int64)


def _model():
    cfg = types.SimpleNamespace(max_source_positions=1500, max_target_positions=448, vocab_size=51865, d_model=128)
    m = types.SimpleNamespace(config=cfg, device=torch.device("cpu"), compute="bf16")
    m.conv_input = lambda feats: feats
    m.encode = lambda x: x[:, :1, :1].reshape(-1, 1).clone()    # the window id the features carry, one row a window
    return m


def _run(monkeypatch, fallback_batch, script):
    monkeypatch.setattr(generation, "_Decoder", _ScriptedDecoder)
    _ScriptedDecoder.script = script
    feats = torch.zeros(1, 80, 6000)
    feats[..., 3000:] = 1.0                                      # window 1 carries id 1
    gc = GenerationConfig(decoder_start_token_id=50258, eos_token_id=EOS, pad_token_id=EOS,
                          no_timestamps_token_id=50363, suppress_tokens=[], lang_to_id={"<|zh|>": 50260})
    trace = []
    out = generation._longform(_model(), gc, feats, None, "zh", "transcribe", None, 40, False, 3000, trace,
                               temperature=(0.0, 0.2, 0.4, 0.6), compression_ratio_threshold=1.35,
                               fallback_batch=fallback_batch)
    return out[0].tolist(), trace


def _script():
    loop = [TS0] + [100, 101] * 20 + [EOS]                      # compression ratio >> 1.35: falls back
    short = [TS0, 100, 101, TS0 + 100, EOS]                      # accepted; finishes first in its batch
    longer = [TS0, 300, 301, 302, 303, 304, 305, 306, 307, TS0 + 150, EOS]
    last = [TS0, 400, 401, TS0 + 50, EOS]
    return {(0, 0.0): loop, (0, 0.2): short, (0, 0.4): longer, (0, 0.6): longer, (1, 0.0): last}


def test_batched_fallback_row_finishing_first_equals_sequential(monkeypatch):
    a, ta = _run(monkeypatch, True, _script())
    b, tb = _run(monkeypatch, False, _script())
    assert any(t["batch"] > 1 for t in ta) and all(t["batch"] == 1 for t in tb)
    assert a == b
    # window 0 accepted at T = 0.2 (its predicted eos cut: not the last window), window 1 at T = 0 (final: eos kept)
    assert a == [TS0, 100, 101, TS0 + 100, TS0, 400, 401, TS0 + 50, EOS]
    assert EOS not in a[:-1]


def test_batched_recordings_stay_together(monkeypatch):
    """HF's batched long-form (generation_whisper.py:785-898): two recordings of different lengths decode their
    current windows as ONE batch per seek iteration; the failing row alone falls back (its remaining temperatures
    speculatively batched), the finished recording leaves the batch, and each recording's tokens are what it gets
    decoded on its own."""
    monkeypatch.setattr(generation, "_Decoder", _ScriptedDecoder)
    script = _script()
    script[(2, 0.0)] = [TS0, 500, 501, TS0 + 20, EOS]
    _ScriptedDecoder.script = script
    feats = torch.zeros(2, 80, 6000)
    feats[0, :, 3000:] = 1.0                                      # recording 0: windows 0, 1
    feats[1] = 2.0                                                # recording 1: one 25 s window (id 2)
    mask = torch.ones(2, 6000, dtype=torch.long)
    mask[1, 2500:] = 0
    gc = GenerationConfig(decoder_start_token_id=50258, eos_token_id=EOS, pad_token_id=EOS,
                          no_timestamps_token_id=50363, suppress_tokens=[], lang_to_id={"<|zh|>": 50260})
    trace = []
    out = generation._longform(_model(), gc, feats, mask, "zh", "transcribe", None, 40, False, 3000, trace,
                               temperature=(0.0, 0.2, 0.4, 0.6), compression_ratio_threshold=1.35)
    assert out[0].tolist() == [TS0, 100, 101, TS0 + 100, TS0, 400, 401, TS0 + 50, EOS]
    assert out[1].tolist()[:5] == [TS0, 500, 501, TS0 + 20, EOS] and set(out[1].tolist()[5:]) <= {EOS}
    first = [t for t in trace if t["T"] == 0.0 and t["seek"] == 0]
    assert [t["b"] for t in first] == [0, 1] and all(t["batch"] == 2 for t in first)
    fb = [t for t in trace if t["T"] > 0]
    assert {t["b"] for t in fb} == {0} and all(t["batch"] == 4 for t in fb)     # 3 temperatures, padded to 4 rows
    later = [t for t in trace if t["seek"] > 0]
    assert [t["b"] for t in later] == [0] and later[0]["batch"] == 1            # recording 1 left the batch
    solo0, _ = _run(monkeypatch, True, _script())
    assert out[0].tolist() == solo0


def test_batched_recordings_empty_and_level_by_level(monkeypatch):
    """A recording of length 0 never enters the batch (HF: seek >= max_frames from the start) and comes back as an
    all-pad row; fallback_batch=False decodes the failing rows level by level (one temperature per decode), with the
    same tokens as the speculative form."""
    monkeypatch.setattr(generation, "_Decoder", _ScriptedDecoder)
    script = _script()
    script[(2, 0.0)] = [TS0, 500, 501, TS0 + 20, EOS]
    feats = torch.zeros(3, 80, 6000)
    feats[0, :, 3000:] = 1.0
    feats[2] = 2.0
    mask = torch.ones(3, 6000, dtype=torch.long)
    mask[1] = 0                                                    # recording 1: empty
    mask[2, 2500:] = 0
    gc = GenerationConfig(decoder_start_token_id=50258, eos_token_id=EOS, pad_token_id=EOS,
                          no_timestamps_token_id=50363, suppress_tokens=[], lang_to_id={"<|zh|>": 50260})
    outs = []
    for fb in (True, False):
        _ScriptedDecoder.script = script
        trace = []
        out = generation._longform(_model(), gc, feats, mask, "zh", "transcribe", None, 40, False, 3000, trace,
                                   temperature=(0.0, 0.2, 0.4, 0.6), compression_ratio_threshold=1.35,
                                   fallback_batch=fb)
        assert 1 not in {t["b"] for t in trace}
        assert set(out[1].tolist()) == {EOS}
        if not fb:
            assert all(t["batch"] <= 2 for t in trace)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


def test_row_tokens():
    assert generation.row_tokens([1, 2, EOS, EOS, EOS], EOS) == [1, 2, EOS]
    assert generation.row_tokens([1, 2, 3], EOS) == [1, 2, 3]
    assert generation.row_tokens([EOS, EOS], EOS) == [EOS]


@pytest.mark.parametrize("compute,batched", [("bf16", True), ("fp16", True), ("fp32", False)])
def test_fallback_batch_only_where_rows_are_independent(monkeypatch, compute, batched):
    monkeypatch.setattr(generation, "_Decoder", _ScriptedDecoder)
    _ScriptedDecoder.script = _script()
    m = _model()
    m.compute = compute
    feats = torch.zeros(1, 80, 6000)
    feats[..., 3000:] = 1.0
    gc = GenerationConfig(eos_token_id=EOS, pad_token_id=EOS, lang_to_id={"<|zh|>": 50260})
    trace = []
    generation._longform(m, gc, feats, None, "zh", "transcribe", None, 40, False, 3000, trace,
                         temperature=(0.0, 0.2, 0.4, 0.6), compression_ratio_threshold=1.35, fallback_batch=True)
    assert any(t["batch"] > 1 for t in trace) == batched


@pytest.mark.parametrize("ngen", [0, 1, 2, 5])
def test_beam_timestamp_rules_match_oracle(ngen):
    """The beam decoder's vectorised HF WhisperTimeStampLogitsProcessor (generation._BeamDecoder._ts_rules, applied
    to the B*k processed log-prob rows) masks exactly what the per-row oracle restatement (oracle/greedy_ref.py
    timestamp_rules) masks, for histories with text, single and paired timestamps, at the first step and later;
    some rows carry enough timestamp mass to trigger the "timestamps beat every text token" rule."""
    from oracle.greedy_ref import timestamp_rules
    V, tb, no_ts, eos, P, mi = 51865, 50364, 50363, 50257, 3, 50
    B, nb = 3, 4
    g = torch.Generator().manual_seed(17 + ngen)
    run_seq = torch.full((B, nb, P + 12), 50257, dtype=torch.int64)
    run_seq[:, :, :P] = torch.tensor([50258, 50260, 50359])
    last_ts = torch.full((B, nb), -1, dtype=torch.int64)
    gens = []
    for r in range(B * nb):
        gen, t_last = [], tb
        for i in range(ngen):
            kind = int(torch.randint(0, 3, (1,), generator=g))
            if kind == 0 or (i > 0 and gen[-1] >= tb and (i < 2 or gen[-2] >= tb)):
                tok = int(torch.randint(0, eos, (1,), generator=g))          # text
            else:
                t_last = t_last + int(torch.randint(0, 30, (1,), generator=g))
                tok = t_last                                                    # a non-decreasing timestamp
            gen.append(tok)
        gens.append(gen)
        run_seq[r // nb, r % nb, P:P + ngen] = torch.tensor(gen, dtype=torch.int64)
        stamps = [t for t in gen if t >= tb]
        last_ts[r // nb, r % nb] = stamps[-1] if stamps else -1
    logits = torch.randn(B * nb, V, generator=g) * 3
    logits[::3, tb:] += 6.0                                                     # timestamp-heavy rows
    logp = torch.log_softmax(logits, -1)
    ns = types.SimpleNamespace(ts=(tb, no_ts, mi), eos=eos, P=P)
    got = generation._BeamDecoder._ts_rules(ns, logp.clone(), run_seq, last_ts, P + ngen)
    for r in range(B * nb):
        want = timestamp_rules(logp[r], gens[r], ngen == 0, ts_begin=tb, no_ts=no_ts, eos=eos, max_initial=mi)
        assert torch.equal(torch.isinf(got[r]), torch.isinf(want)), (r, gens[r])
        fin = ~torch.isinf(want)
        assert torch.equal(got[r][fin], want[fin]), r
