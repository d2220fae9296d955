"""Self-contained WAV reader/writer (librosa/soundfile are not available offline).

* ``read_audio(path, sr=44100)`` -- stands in for ``librosa.load(path, sr=44100, mono=False)``
  (inference_pytorch.py:213): float32 [channels, samples] scaled like soundfile (PCM / 2^(bits-1)),
  resampled with scipy's polyphase filter when the file rate differs (librosa's default soxr
  filter differs in the last bits; documented divergence).
* ``write_audio(path, data[samples, channels], sr, subtype)`` -- ``sf.write`` for WAV with subtype
  FLOAT / PCM_16 / PCM_24 (inference_pytorch.py:262-272; ensemble.py:311 uses PCM_24).
"""
import struct
from fractions import Fraction

import numpy as np

_PCM, _FLOAT, _EXT = 1, 3, 0xFFFE


def read_wav(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
            if fmt[0] == _EXT and len(body) >= 26:
                fmt = (struct.unpack("<H", body[24:26])[0],) + fmt[1:]
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    tag, ch, sr, _, align, bits = fmt
    n = len(payload) // align
    if tag == _FLOAT and bits == 32:
        x = np.frombuffer(payload[:n * align], "<f4").astype(np.float32)
    elif tag == _FLOAT and bits == 64:
        x = np.frombuffer(payload[:n * align], "<f8").astype(np.float32)
    elif tag == _PCM and bits == 16:
        x = np.frombuffer(payload[:n * align], "<i2").astype(np.float32) / 32768.0
    elif tag == _PCM and bits == 24:
        b = np.frombuffer(payload[:n * align], np.uint8).reshape(-1, 3).astype(np.int32)
        v = (b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16))
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / 8388608.0
    elif tag == _PCM and bits == 32:
        x = np.frombuffer(payload[:n * align], "<i4").astype(np.float64) / 2147483648.0
        x = x.astype(np.float32)
    elif tag == _PCM and bits == 8:
        x = (np.frombuffer(payload[:n * align], np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"{path}: unsupported WAV format tag={tag} bits={bits}")
    return x.reshape(n, ch).T.copy(), sr


def read_audio(path, sr=44100):
    x, file_sr = read_wav(path)
    if sr is not None and file_sr != sr:
        from scipy.signal import resample_poly
        fr = Fraction(sr, file_sr).limit_denominator(1000)
        x = resample_poly(x, fr.numerator, fr.denominator, axis=-1).astype(np.float32)
        file_sr = sr
    return x, file_sr


def write_audio(path, data, sr, subtype="FLOAT"):
    """data: [samples, channels] (soundfile orientation)."""
    data = np.asarray(data)
    if data.ndim == 1:
        data = data[:, None]
    n, ch = data.shape
    if subtype == "FLOAT":
        tag, bits, payload = _FLOAT, 32, data.astype("<f4").tobytes()
    elif subtype == "PCM_16":
        v = np.clip(np.round(data * 32768.0), -32768, 32767).astype("<i2")
        tag, bits, payload = _PCM, 16, v.tobytes()
    elif subtype == "PCM_24":
        v = np.clip(np.round(data * 8388608.0), -8388608, 8388607).astype(np.int32).reshape(-1)
        b = np.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], -1).astype(np.uint8)
        tag, bits, payload = _PCM, 24, b.tobytes()
    else:
        raise ValueError(f"unsupported subtype {subtype}")
    align = ch * bits // 8
    fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * align, align, bits)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(payload)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt)
        f.write(b"data" + struct.pack("<I", len(payload)) + payload)
