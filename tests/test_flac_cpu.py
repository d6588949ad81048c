"""Native FLAC decoding for the data feed (csrc/flac.cpp via tw.dataset.read_audio / decode_flac): the
reference reads its corpus with soundfile (dataset/cool_dataset.py:55, `.flac`), absent in this image.

Pinning: (1) the example file published in RFC 9639 (Appendix D.1, written by libFLAC): its two samples
decode to values whose MD5 equals the MD5 libFLAC stored in STREAMINFO, and both frame CRCs check;
(2) round trips through a spec-restated test encoder (tests/flac_encoder.py) over every construct the
decoder reads -- subframe kinds, predictor orders, Rice partition orders / parameter widths / escapes,
wasted bits, stereo decorrelation modes, header codings, bit depths -- bit-exact, and the decoded MD5
equals the encoder's STREAMINFO MD5; (3) corrupted or truncated streams raise."""
import hashlib
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "taiwan-whisper_amd"))
sys.path.insert(0, HERE)

import flac_encoder as fe  # noqa: E402

# RFC 9639 Appendix D.1 (decoding example 1): 44.1 kHz, 16-bit stereo, one sample
RFC_D1 = bytes.fromhex("664c61438000002210001000" "00000f00000f0ac442f00000" "00013e84b41807dc69030758"
                       "6a3dad1a2e0ffff869180000" "bf0358fd03128baa9a")


def _ints(y, bps):
    return np.round(np.asarray(y) * (1 << (bps - 1))).astype(np.int64)


def _md5(s, bps):
    nb = (bps + 7) // 8
    return hashlib.md5(b"".join(int(v).to_bytes(nb, "little", signed=True) for v in np.asarray(s).reshape(-1))).digest()


def test_rfc9639_example_1():
    from tw.dataset import decode_flac
    y, sr = decode_flac(RFC_D1)
    s = _ints(y, 16)
    assert sr == 44100 and s.tolist() == [[25588, 10416]]
    assert _md5(s, 16) == RFC_D1[26:42]


def _signal(n, ch, bps, seed, kind="tone"):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) * 0.4
    cols = []
    for c in range(ch):
        if kind == "tone":
            v = amp * np.sin(2 * np.pi * (220 + 97 * c) * t / 16000) + rng.normal(0, amp / 200, n)
        elif kind == "noise":
            v = rng.normal(0, amp / 3, n)
        elif kind == "wasted":
            v = np.round(amp * np.sin(2 * np.pi * 300 * t / 16000) / 8) * 8
        else:
            v = np.full(n, (c + 1) * 100.0)
        cols.append(np.clip(np.round(v), -(1 << (bps - 1)), (1 << (bps - 1)) - 1))
    return np.stack(cols, 1).astype(np.int64)


CASES = [
    dict(ch=1, bps=16, kinds=("verbatim", "fixed0", "fixed1", "fixed2", "fixed3", "fixed4", "lpc", "constant")),
    dict(ch=1, bps=16, kinds=("fixed2",), porder=4, method=1),
    dict(ch=1, bps=16, kinds=("lpc",), porder=2, escape_part=1),
    dict(ch=2, bps=16, kinds=("fixed2", "lpc"), stereo="left_side"),
    dict(ch=2, bps=16, kinds=("fixed1", "lpc"), stereo="side_right"),
    dict(ch=2, bps=16, kinds=("fixed3", "lpc"), stereo="mid_side", porder=3),
    dict(ch=2, bps=24, kinds=("lpc", "fixed2"), stereo="mid_side", sample_rate=48000),
    dict(ch=1, bps=24, kinds=("fixed4",), method=1, porder=5),
    dict(ch=1, bps=8, kinds=("fixed1", "verbatim"), sample_rate=22050),
    dict(ch=1, bps=16, kinds=("fixed2",), signal="wasted"),
    dict(ch=2, bps=16, kinds=("constant",), signal="const"),
    dict(ch=1, bps=16, kinds=("lpc",), signal="noise", block_size=1152),
    dict(ch=1, bps=16, kinds=("fixed2",), sample_rate=16000, header_rate_code="explicit", header_bs_code="explicit"),
    dict(ch=1, bps=16, kinds=("fixed2",), sample_rate=16000, header_rate_code="hz"),
    dict(ch=1, bps=16, kinds=("fixed2",), header_rate_code="streaminfo"),
    dict(ch=3, bps=16, kinds=("fixed2",)),
    dict(ch=1, bps=16, kinds=("fixed2",), id3=True),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_round_trip(case):
    from tw.dataset import decode_flac
    c = dict(CASES[case])
    ch, bps = c.pop("ch"), c["bps"]
    n = 16000 * 2 + 1234                       # a short last block (odd size: 8/16-bit block-size codes)
    x = _signal(n, ch, bps, case, c.pop("signal", "tone"))
    data = fe.encode(x if ch > 1 else x[:, 0], **c)
    y, sr = decode_flac(data)
    assert sr == c.get("sample_rate", 16000)
    s = _ints(y, bps)
    assert np.array_equal(s.reshape(n, ch), x)
    assert _md5(s, bps) == data[data.index(b"fLaC") + 4 + 4 + 18: data.index(b"fLaC") + 4 + 4 + 34]


def test_corrupt_and_truncated_streams_raise():
    from tw.dataset import decode_flac
    x = _signal(9000, 1, 16, 7)[:, 0]
    data = bytearray(fe.encode(x, kinds=("fixed2",)))
    bad = bytearray(data)
    bad[len(bad) // 2] ^= 0x10                  # inside a frame: CRC-16 (or a header CRC-8) fails
    with pytest.raises(RuntimeError):
        decode_flac(bytes(bad))
    with pytest.raises(RuntimeError):
        decode_flac(bytes(data[: len(data) - 5]))
    with pytest.raises(RuntimeError):
        decode_flac(b"RIFF" + bytes(data[4:]))


def test_read_audio_flac_matches_wav(tmp_path):
    """read_audio(.flac) == read_audio(.wav) of the same PCM (the soundfile scaling), and the NTU-COOL
    dataset reads a .flac clip with its 5-line transcript."""
    import wave
    from tw.dataset import CoolDataset, read_audio
    x = _signal(16000 * 3, 1, 16, 3)[:, 0]
    (tmp_path / "a.flac").write_bytes(fe.encode(x, kinds=("lpc",)))
    with wave.open(str(tmp_path / "a.wav"), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(x.astype("<i2").tobytes())
    a, sa = read_audio(str(tmp_path / "a.flac"))
    b, sb = read_audio(str(tmp_path / "a.wav"))
    assert sa == sb == 16000 and np.array_equal(a, b)
    (tmp_path / "a.txt").write_text("0.00\n3.00\n你好\n<|0.00|>你好<|3.00|>\n\n")
    man = tmp_path / "m.tsv"
    man.write_text(f"{tmp_path}\na.flac\n")
    ds = CoolDataset(str(man))
    item = ds[0]
    assert item["audio"]["sampling_rate"] == 16000 and np.array_equal(item["audio"]["array"], a)
