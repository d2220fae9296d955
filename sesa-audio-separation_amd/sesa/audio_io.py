"""Self-contained audio reader/writer (librosa/soundfile are not available offline).

* ``read_audio(path, sr=44100)`` -- stands in for ``librosa.load(path, sr=44100, mono=False)``
  (inference_pytorch.py:213) for WAV (PCM 8/16/24/32, float 32/64) and FLAC (libsesa's FLAC decoder,
  csrc/sesa_flac.cpp): float32 [channels, samples] scaled like soundfile (int / 2^(bits-1)),
  resampled with scipy's polyphase filter when the file rate differs (librosa's default soxr filter
  differs in the last bits; documented divergence).  Other containers (mp3, ogg, m4a, aac) have no
  offline decoder here and raise.
* ``write_audio(path, data[samples, channels], sr, subtype)`` -- ``sf.write``: ``.flac`` paths are
  FLAC (PCM_16 / PCM_24), anything else WAV (FLOAT / PCM_16 / PCM_24) (inference_pytorch.py:262-272;
  ensemble.py:311 uses PCM_24).  float -> PCM as libsndfile's write path: ``lrintf(x * (2^(bits-1)
  - 1))`` in float32 without clipping for WAV (out-of-range samples wrap exactly as libsndfile's
  non-clipping conversion does); FLAC clips (libFLAC cannot store wider values).
"""
import ctypes
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


def _lib():
    from . import _native as N
    return N


def flac_max_samples(data, channels):
    """Upper bound on the samples per channel a FLAC stream of ``len(data)`` bytes can decode to
    (RFC 9639): every frame holds at most STREAMINFO's maximum block size and takes at least a
    6-byte header, a 2-byte CRC-16 and a 2-byte CONSTANT subframe per channel.  Guards the
    preallocation against a corrupt or hostile 36-bit total_samples."""
    max_block = struct.unpack(">H", data[10:12])[0] if len(data) >= 12 else 65535
    min_frame = 6 + 2 + 2 * max(1, channels)
    return (len(data) // min_frame + 1) * max(16, max_block or 65535)


def read_flac(path):
    N = _lib()
    with open(path, "rb") as f:
        data = f.read()
    buf = ctypes.create_string_buffer(data, len(data))
    ch, sr, bits, frames = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    N.check(N.lib().sesa_flac_info(buf, len(data), ctypes.byref(ch), ctypes.byref(sr), ctypes.byref(bits),
                                   ctypes.byref(frames)), f"FLAC {path}")
    bound = flac_max_samples(data, ch.value)
    if frames.value < 0 or frames.value > bound:
        raise ValueError(f"FLAC {path}: STREAMINFO declares {frames.value} samples, more than the "
                         f"{len(data)}-byte file can hold (<= {bound}); corrupt header")
    out = np.zeros((frames.value, ch.value), np.float32)
    got = ctypes.c_int64()
    N.check(N.lib().sesa_flac_decode(buf, len(data), out.ctypes.data, frames.value, ctypes.byref(got)),
            f"FLAC {path}")
    return out[:got.value].T.copy(), sr.value


def read_any(path):
    with open(path, "rb") as f:
        magic = f.read(4)
    if magic == b"fLaC":
        return read_flac(path)
    if magic == b"RIFF":
        return read_wav(path)
    raise ValueError(f"{path}: unsupported container (WAV and FLAC only offline; no mp3/ogg/m4a decoder)")


def read_audio(path, sr=44100):
    x, file_sr = read_any(path)
    if sr is not None and file_sr != sr:
        from scipy.signal import resample_poly
        fr = Fraction(sr, file_sr).limit_denominator(1000)
        x = resample_poly(x, fr.numerator, fr.denominator, axis=-1).astype(np.float32)
        file_sr = sr
    return x, file_sr


def quantize_pcm(data, bits, clip=False):
    """libsndfile float -> PCM (pcm.c f2s / f2let, normalisation on): lrintf(x * (2^(bits-1) - 1)) in
    float32, round half to even; without clipping the integer wraps like the C cast."""
    scale = np.float32(2 ** (bits - 1) - 1)
    v = np.rint(np.asarray(data, np.float32) * scale).astype(np.int64)
    if clip:
        return np.clip(v, -(1 << (bits - 1)), (1 << (bits - 1)) - 1)
    m = 1 << bits
    return ((v + (m >> 1)) % m) - (m >> 1)


def write_flac(path, data, sr, subtype):
    N = _lib()
    bits = {"PCM_16": 16, "PCM_24": 24}.get(subtype)
    if bits is None:
        raise ValueError(f"FLAC supports PCM_16 / PCM_24, not {subtype}")
    x = np.ascontiguousarray(np.asarray(data, np.float32))
    if x.ndim == 1:
        x = x[:, None]
    n, ch = x.shape
    cap = N.lib().sesa_flac_encode_bound(n, ch, bits)
    out = ctypes.create_string_buffer(cap)
    w = ctypes.c_size_t()
    N.check(N.lib().sesa_flac_encode(x.ctypes.data, n, ch, int(sr), bits, out, cap, ctypes.byref(w)), "FLAC encode")
    with open(path, "wb") as f:
        f.write(out.raw[:w.value])


def write_audio(path, data, sr, subtype="FLOAT"):
    """data: [samples, channels] (soundfile orientation); ``.flac`` -> FLAC, else WAV."""
    if str(path).lower().endswith(".flac"):
        return write_flac(path, data, sr, subtype)
    data = np.asarray(data)
    if data.ndim == 1:
        data = data[:, None]
    n, ch = data.shape
    if subtype == "FLOAT":
        tag, bits, payload = _FLOAT, 32, data.astype("<f4").tobytes()
    elif subtype == "PCM_16":
        tag, bits, payload = _PCM, 16, quantize_pcm(data, 16).astype("<i2").tobytes()
    elif subtype == "PCM_24":
        v = quantize_pcm(data, 24).astype(np.int64).reshape(-1)
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
