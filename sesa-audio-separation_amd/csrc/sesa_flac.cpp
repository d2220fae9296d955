// FLAC codec (host) for the CLI's audio I/O: the reference reads inputs with librosa.load
// (inference_pytorch.py:213, any libsndfile format incl. FLAC) and writes stems with
// sf.write(..., subtype=PCM_16 / PCM_24) into <name>_<instr>.flac when --flac_file (:262-272).
// libsndfile / libFLAC are not in this image, so the format is implemented here from the FLAC
// specification (RFC 9639):
//   decoder -- every subframe type (CONSTANT, VERBATIM, FIXED 0-4, LPC 1-32), Rice / Rice2 residuals
//              with escapes, wasted bits, all stereo decorrelations, fixed or variable blocking,
//              frame CRC-8 / CRC-16 checked; samples scaled like libsndfile's float read (/ 2^(bps-1))
//   encoder -- fixed blocking (4096), per channel the best of CONSTANT / FIXED order 0-4 / VERBATIM,
//              partitioned Rice residuals; float -> int as libsndfile's float write (x * (2^(bps-1)-1),
//              round half to even) clipped to the bps range (libFLAC cannot store wider values)
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "sesa_common.hpp"

namespace sesa {
namespace {

uint8_t crc8_tab[256];
uint16_t crc16_tab[256];
struct CrcInit {
  CrcInit() {
    for (int i = 0; i < 256; ++i) {
      uint8_t c = (uint8_t)i;
      for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
      crc8_tab[i] = c;
      uint16_t d = (uint16_t)(i << 8);
      for (int b = 0; b < 8; ++b) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : d << 1);
      crc16_tab[i] = d;
    }
  }
} crc_init;

uint8_t crc8(const uint8_t* p, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; ++i) c = crc8_tab[c ^ p[i]];
  return c;
}
uint16_t crc16(const uint8_t* p, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; ++i) c = (uint16_t)((c << 8) ^ crc16_tab[(c >> 8) ^ p[i]]);
  return c;
}

// ---- decoder ----------------------------------------------------------------------------------
struct BitReader {
  const uint8_t* p;
  size_t n, pos = 0;  // bit position
  bool bad = false;
  BitReader(const uint8_t* d, size_t len) : p(d), n(len * 8) {}
  uint64_t bits(int k) {  // k <= 57
    if (k == 0) return 0;
    if (pos + k > n) {
      bad = true;
      pos = n;
      return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < k;) {
      const size_t byte = pos >> 3;
      const int off = (int)(pos & 7);
      const int take = std::min(8 - off, k - i);
      const uint32_t b = (p[byte] >> (8 - off - take)) & ((1u << take) - 1);
      v = (v << take) | b;
      pos += take;
      i += take;
    }
    return v;
  }
  int64_t sbits(int k) {
    if (k == 0) return 0;
    const uint64_t v = bits(k);
    return (int64_t)(v << (64 - k)) >> (64 - k);
  }
  uint32_t unary() {  // count of 0 bits before a 1
    uint32_t q = 0;
    while (!bad) {
      if (pos >= n) {
        bad = true;
        break;
      }
      const size_t byte = pos >> 3;
      const int off = (int)(pos & 7);
      const uint8_t rest = (uint8_t)(p[byte] << off);
      if (rest == 0) {
        q += 8 - off;
        pos += 8 - off;
        continue;
      }
      const int lz = __builtin_clz((uint32_t)rest) - 24;
      q += lz;
      pos += lz + 1;
      break;
    }
    return q;
  }
  void align() { pos = (pos + 7) & ~(size_t)7; }
  size_t byte_pos() const { return pos >> 3; }
};

struct StreamInfo {
  int min_block = 0, max_block = 0, rate = 0, channels = 0, bps = 0;
  int64_t total = 0;
  size_t first_frame = 0;
};

int parse_header(const uint8_t* d, size_t n, StreamInfo* si) {
  SESA_REQUIRE(n >= 42 && memcmp(d, "fLaC", 4) == 0, SESA_ERR_INVALID, "flac: not a FLAC stream (no fLaC marker)");
  size_t pos = 4;
  bool last = false, have_info = false;
  while (!last) {
    SESA_REQUIRE(pos + 4 <= n, SESA_ERR_INVALID, "flac: truncated metadata");
    last = (d[pos] & 0x80) != 0;
    const int type = d[pos] & 0x7f;
    const size_t len = ((size_t)d[pos + 1] << 16) | ((size_t)d[pos + 2] << 8) | d[pos + 3];
    pos += 4;
    SESA_REQUIRE(pos + len <= n, SESA_ERR_INVALID, "flac: truncated metadata block");
    if (type == 0) {
      SESA_REQUIRE(len >= 34, SESA_ERR_INVALID, "flac: short STREAMINFO");
      BitReader br(d + pos, len);
      si->min_block = (int)br.bits(16);
      si->max_block = (int)br.bits(16);
      br.bits(24);
      br.bits(24);
      si->rate = (int)br.bits(20);
      si->channels = (int)br.bits(3) + 1;
      si->bps = (int)br.bits(5) + 1;
      si->total = (int64_t)br.bits(36);
      have_info = true;
    }
    pos += len;
  }
  SESA_REQUIRE(have_info, SESA_ERR_INVALID, "flac: missing STREAMINFO");
  SESA_REQUIRE(si->bps >= 4 && si->bps <= 32, SESA_ERR_INVALID, "flac: unsupported bits per sample %d", si->bps);
  si->first_frame = pos;
  return SESA_OK;
}

bool read_utf8(BitReader& br, uint64_t* v) {
  const uint32_t b0 = (uint32_t)br.bits(8);
  int extra = 0;
  uint64_t val;
  if (!(b0 & 0x80)) {
    val = b0;
  } else if ((b0 & 0xE0) == 0xC0) {
    val = b0 & 0x1F; extra = 1;
  } else if ((b0 & 0xF0) == 0xE0) {
    val = b0 & 0x0F; extra = 2;
  } else if ((b0 & 0xF8) == 0xF0) {
    val = b0 & 0x07; extra = 3;
  } else if ((b0 & 0xFC) == 0xF8) {
    val = b0 & 0x03; extra = 4;
  } else if ((b0 & 0xFE) == 0xFC) {
    val = b0 & 0x01; extra = 5;
  } else if (b0 == 0xFE) {
    val = 0; extra = 6;
  } else {
    return false;
  }
  for (int i = 0; i < extra; ++i) {
    const uint32_t b = (uint32_t)br.bits(8);
    if ((b & 0xC0) != 0x80) return false;
    val = (val << 6) | (b & 0x3F);
  }
  *v = val;
  return !br.bad;
}

bool decode_residual(BitReader& br, int block, int order, int64_t* res) {
  const int method = (int)br.bits(2);
  if (method > 1) return false;
  const int pbits = method == 0 ? 4 : 5;
  const uint32_t esc = method == 0 ? 15u : 31u;
  const int porder = (int)br.bits(4);
  const int parts = 1 << porder;
  if ((block >> porder) < order || (block & (parts - 1))) return false;
  int i = order;
  for (int p = 0; p < parts; ++p) {
    const int cnt = (block >> porder) - (p == 0 ? order : 0);
    const uint32_t k = (uint32_t)br.bits(pbits);
    if (k == esc) {
      const int nb = (int)br.bits(5);
      for (int j = 0; j < cnt; ++j) res[i++] = br.sbits(nb);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = br.unary();
        const uint64_t u = (q << k) | br.bits((int)k);
        res[i++] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
      }
    }
    if (br.bad) return false;
  }
  return true;
}

bool decode_subframe(BitReader& br, int block, int bps, int64_t* s) {
  if (br.bits(1) != 0) return false;
  const int type = (int)br.bits(6);
  int wasted = 0;
  if (br.bits(1)) wasted = (int)br.unary() + 1;
  bps -= wasted;
  if (bps <= 0 || bps > 33) return false;
  if (type == 0) {
    const int64_t v = br.sbits(bps);
    for (int i = 0; i < block; ++i) s[i] = v;
  } else if (type == 1) {
    for (int i = 0; i < block; ++i) s[i] = br.sbits(bps);
  } else if (type >= 8 && type <= 12) {
    const int order = type - 8;
    if (order > block) return false;
    for (int i = 0; i < order; ++i) s[i] = br.sbits(bps);
    if (!decode_residual(br, block, order, s)) return false;
    for (int i = order; i < block; ++i) {
      int64_t pred = 0;
      switch (order) {
        case 1: pred = s[i - 1]; break;
        case 2: pred = 2 * s[i - 1] - s[i - 2]; break;
        case 3: pred = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
        case 4: pred = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
        default: break;
      }
      s[i] += pred;
    }
  } else if (type >= 32) {
    const int order = type - 31;
    if (order > block) return false;
    for (int i = 0; i < order; ++i) s[i] = br.sbits(bps);
    const int prec = (int)br.bits(4) + 1;
    if (prec == 16) return false;
    const int shift = (int)br.sbits(5);
    if (shift < 0) return false;
    int64_t coef[32];
    for (int i = 0; i < order; ++i) coef[i] = br.sbits(prec);
    if (!decode_residual(br, block, order, s)) return false;
    for (int i = order; i < block; ++i) {
      int64_t acc = 0;
      for (int j = 0; j < order; ++j) acc += coef[j] * s[i - 1 - j];
      s[i] += acc >> shift;
    }
  } else {
    return false;
  }
  if (wasted)
    for (int i = 0; i < block; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return !br.bad;
}

// Decodes every frame; calls sink(block, channels, samples[ch][block]) per frame.
template <class Sink>
int decode_frames(const uint8_t* d, size_t n, const StreamInfo& si, Sink sink) {
  static const int rates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
  static const int sizes[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  size_t pos = si.first_frame;
  std::vector<int64_t> buf;
  while (pos + 2 <= n) {
    // resynchronise on the 14-bit frame sync code
    if (!(d[pos] == 0xFF && (d[pos + 1] & 0xFE) == 0xF8)) {
      ++pos;
      continue;
    }
    BitReader br(d + pos, n - pos);
    br.bits(15);
    br.bits(1);  // blocking strategy (frame vs sample number: both decoded the same way here)
    const int bcode = (int)br.bits(4);
    const int rcode = (int)br.bits(4);
    const int ccode = (int)br.bits(4);
    const int scode = (int)br.bits(3);
    br.bits(1);
    uint64_t num;
    if (!read_utf8(br, &num) || bcode == 0 || rcode == 15 || ccode > 10 || scode == 3) {
      ++pos;
      continue;
    }
    int block;
    if (bcode == 1) block = 192;
    else if (bcode <= 5) block = 576 << (bcode - 2);
    else if (bcode == 6) block = (int)br.bits(8) + 1;
    else if (bcode == 7) block = (int)br.bits(16) + 1;
    else block = 256 << (bcode - 8);
    if (rcode == 12) br.bits(8);
    else if (rcode == 13 || rcode == 14) br.bits(16);
    const size_t hdr_bytes = br.byte_pos();
    const uint8_t c8 = (uint8_t)br.bits(8);
    if (br.bad || crc8(d + pos, hdr_bytes) != c8) {
      ++pos;
      continue;
    }
    (void)rates;
    const int bps = scode ? sizes[scode] : si.bps;
    const int nch = ccode <= 7 ? ccode + 1 : 2;
    SESA_REQUIRE(nch == si.channels, SESA_ERR_INVALID, "flac: frame channel count %d != STREAMINFO %d", nch,
                 si.channels);
    buf.assign((size_t)nch * block, 0);
    bool ok = true;
    for (int c = 0; c < nch && ok; ++c) {
      int sb = bps;
      if ((ccode == 8 && c == 1) || (ccode == 9 && c == 0) || (ccode == 10 && c == 1)) sb += 1;  // side channel
      ok = decode_subframe(br, block, sb, buf.data() + (size_t)c * block);
    }
    br.align();
    const size_t frame_end = br.byte_pos();
    const uint16_t c16 = (uint16_t)br.bits(16);
    if (!ok || br.bad || crc16(d + pos, frame_end) != c16) {
      ++pos;
      continue;
    }
    int64_t* a = buf.data();
    int64_t* b = buf.data() + block;
    if (ccode == 8) {
      for (int i = 0; i < block; ++i) b[i] = a[i] - b[i];
    } else if (ccode == 9) {
      for (int i = 0; i < block; ++i) a[i] += b[i];
    } else if (ccode == 10) {
      for (int i = 0; i < block; ++i) {
        const int64_t side = b[i];
        const int64_t mid = ((uint64_t)a[i] << 1) | (side & 1);
        a[i] = (mid + side) >> 1;
        b[i] = (mid - side) >> 1;
      }
    }
    const int rc = sink(block, nch, bps, buf.data());
    if (rc) return rc;
    pos += frame_end + 2;
  }
  return SESA_OK;
}

// ---- encoder -----------------------------------------------------------------------------------
struct BitWriter {
  std::vector<uint8_t> out;
  uint64_t acc = 0;
  int nacc = 0;
  void put(uint64_t v, int k) {  // k <= 32
    if (k == 0) return;
    v &= (k == 64) ? ~0ull : ((1ull << k) - 1);
    acc = (acc << k) | v;
    nacc += k;
    while (nacc >= 8) {
      nacc -= 8;
      out.push_back((uint8_t)(acc >> nacc));
    }
  }
  void put_unary(uint32_t q) {  // q zeros then a one
    while (q >= 32) {
      put(0, 32);
      q -= 32;
    }
    put(1, (int)q + 1);
  }
  void align() {
    if (nacc) put(0, 8 - nacc);
  }
};

void put_utf8(BitWriter& bw, uint64_t v) {
  if (v < 0x80) {
    bw.put(v, 8);
    return;
  }
  int extra = v < 0x800 ? 1 : v < 0x10000 ? 2 : v < 0x200000 ? 3 : v < 0x4000000 ? 4 : 5;
  static const uint32_t lead[6] = {0, 0xC0, 0xE0, 0xF0, 0xF8, 0xFC};
  bw.put(lead[extra] | (uint32_t)(v >> (6 * extra)), 8);
  for (int i = extra - 1; i >= 0; --i) bw.put(0x80 | ((v >> (6 * i)) & 0x3F), 8);
}

uint64_t rice_bits(const int64_t* r, int n, int k) {
  uint64_t b = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t u = (uint64_t)((r[i] << 1) ^ (r[i] >> 63));
    b += (u >> k) + 1 + k;
  }
  return b;
}

// best partition order / per-partition Rice parameter for residual r[order..block)
void plan_rice(const int64_t* r, int block, int order, int* best_p, std::vector<int>& ks, uint64_t* best_bits) {
  *best_bits = ~0ull;
  for (int p = 0; p <= 8; ++p) {
    if (block & ((1 << p) - 1)) break;
    if ((block >> p) < order || (block >> p) == 0) break;
    const int parts = 1 << p;
    uint64_t total = 6;  // method + order
    std::vector<int> kk(parts);
    int i = order;
    for (int q = 0; q < parts; ++q) {
      const int cnt = (block >> p) - (q == 0 ? order : 0);
      uint64_t sum = 0;
      for (int j = 0; j < cnt; ++j) sum += (uint64_t)((r[i + j] << 1) ^ (r[i + j] >> 63));
      int k = 0;
      if (cnt > 0) {
        const uint64_t mean = sum / (uint64_t)cnt;
        while (k < 30 && (1ull << (k + 1)) <= mean) ++k;
      }
      uint64_t best = ~0ull;
      int bk = k;
      for (int t = std::max(0, k - 1); t <= std::min(30, k + 1); ++t) {
        const uint64_t b = rice_bits(r + i, cnt, t);
        if (b < best) {
          best = b;
          bk = t;
        }
      }
      kk[q] = bk;
      total += best + 5;  // 5-bit (Rice2) parameter
      i += cnt;
    }
    if (total < *best_bits) {
      *best_bits = total;
      *best_p = p;
      ks = kk;
    }
  }
}

void encode_subframe(BitWriter& bw, const int64_t* s, int block, int bps) {
  bool constant = true;
  for (int i = 1; i < block && constant; ++i) constant = s[i] == s[0];
  if (constant) {
    bw.put(0, 1);
    bw.put(0, 6);
    bw.put(0, 1);
    bw.put((uint64_t)s[0], bps);
    return;
  }
  std::vector<int64_t> r(block), best_r;
  int best_order = -1, best_p = 0;
  std::vector<int> best_k;
  uint64_t best_bits = (uint64_t)block * bps;  // verbatim
  for (int order = 0; order <= 4 && order < block; ++order) {
    for (int i = order; i < block; ++i) {
      int64_t pred = 0;
      switch (order) {
        case 1: pred = s[i - 1]; break;
        case 2: pred = 2 * s[i - 1] - s[i - 2]; break;
        case 3: pred = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
        case 4: pred = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
        default: break;
      }
      r[i] = s[i] - pred;
    }
    int p;
    std::vector<int> ks;
    uint64_t rb;
    plan_rice(r.data(), block, order, &p, ks, &rb);
    const uint64_t total = rb + (uint64_t)order * bps;
    if (total < best_bits) {
      best_bits = total;
      best_order = order;
      best_p = p;
      best_k = ks;
      best_r = r;
    }
  }
  bw.put(0, 1);
  if (best_order < 0) {  // VERBATIM
    bw.put(1, 6);
    bw.put(0, 1);
    for (int i = 0; i < block; ++i) bw.put((uint64_t)s[i], bps);
    return;
  }
  bw.put(8 + best_order, 6);
  bw.put(0, 1);
  for (int i = 0; i < best_order; ++i) bw.put((uint64_t)s[i], bps);
  bw.put(1, 2);  // Rice2 (5-bit parameters)
  bw.put(best_p, 4);
  int i = best_order;
  for (int q = 0; q < (1 << best_p); ++q) {
    const int cnt = (block >> best_p) - (q == 0 ? best_order : 0);
    const int k = best_k[q];
    bw.put(k, 5);
    for (int j = 0; j < cnt; ++j, ++i) {
      const uint64_t u = (uint64_t)((best_r[i] << 1) ^ (best_r[i] >> 63));
      bw.put_unary((uint32_t)(u >> k));
      bw.put(u & ((1ull << k) - 1), k);
    }
  }
}

}  // namespace
}  // namespace sesa

using namespace sesa;

extern "C" int sesa_flac_info(const uint8_t* data, size_t n, int* channels, int* sample_rate, int* bits,
                              int64_t* frames) {
  clear_error();
  SESA_REQUIRE(data && channels && sample_rate && bits && frames, SESA_ERR_INVALID, "flac_info: null argument");
  StreamInfo si;
  const int rc = parse_header(data, n, &si);
  if (rc) return rc;
  *channels = si.channels;
  *sample_rate = si.rate;
  *bits = si.bps;
  if (si.total == 0) {  // unknown length in STREAMINFO: count by decoding
    int64_t cnt = 0;
    const int r2 = decode_frames(data, n, si, [&](int block, int, int, const int64_t*) {
      cnt += block;
      return 0;
    });
    if (r2) return r2;
    si.total = cnt;
  }
  *frames = si.total;
  return SESA_OK;
}

extern "C" int sesa_flac_decode(const uint8_t* data, size_t n, float* out, int64_t max_frames, int64_t* frames_out) {
  clear_error();
  SESA_REQUIRE(data && out && frames_out && max_frames >= 0, SESA_ERR_INVALID, "flac_decode: bad arguments");
  StreamInfo si;
  int rc = parse_header(data, n, &si);
  if (rc) return rc;
  int64_t w = 0;
  rc = decode_frames(data, n, si, [&](int block, int nch, int bps, const int64_t* s) {
    const double scale = 1.0 / (double)(1ll << (bps - 1));
    for (int i = 0; i < block && w < max_frames; ++i, ++w)
      for (int c = 0; c < nch; ++c) out[w * nch + c] = (float)((double)s[(size_t)c * block + i] * scale);
    return 0;
  });
  *frames_out = w;
  return rc;
}

extern "C" size_t sesa_flac_encode_bound(int64_t frames, int channels, int bits) {
  if (frames < 0 || channels < 1 || bits < 4) return 0;
  const int64_t blocks = (frames + 4095) / 4096;
  return (size_t)(42 + blocks * (32 + channels * 2) + (frames * channels * (bits + 1)) / 8 + 64);
}

extern "C" int sesa_flac_encode(const float* in, int64_t frames, int channels, int sample_rate, int bits,
                                uint8_t* out, size_t cap, size_t* written) {
  clear_error();
  SESA_REQUIRE(in && out && written && frames >= 0 && channels >= 1 && channels <= 8, SESA_ERR_INVALID,
               "flac_encode: bad arguments");
  SESA_REQUIRE(bits == 16 || bits == 24, SESA_ERR_INVALID, "flac_encode: PCM_16 / PCM_24 only");
  SESA_REQUIRE(sample_rate > 0 && sample_rate < (1 << 20), SESA_ERR_INVALID, "flac_encode: sample rate");
  const int B = 4096;
  BitWriter bw;
  bw.out.insert(bw.out.end(), {'f', 'L', 'a', 'C'});
  bw.put(0x80, 8);  // last metadata block, STREAMINFO
  bw.put(34, 24);
  bw.put(frames < B ? (frames > 16 ? frames : 16) : B, 16);
  bw.put(B, 16);
  bw.put(0, 24);
  bw.put(0, 24);
  bw.put(sample_rate, 20);
  bw.put(channels - 1, 3);
  bw.put(bits - 1, 5);
  bw.put((uint64_t)frames >> 4, 32);
  bw.put((uint64_t)frames & 15, 4);
  for (int i = 0; i < 16; ++i) bw.put(0, 8);  // MD5 unknown
  // float -> int as libsndfile's write path: x * (2^(bits-1) - 1) in float, round half to even
  const float scale = bits == 16 ? 32767.0f : 8388607.0f;
  const int64_t lo = -(1ll << (bits - 1)), hi = (1ll << (bits - 1)) - 1;
  int rcode = sample_rate == 44100 ? 9 : sample_rate == 48000 ? 10 : sample_rate == 96000 ? 11 : 0;
  std::vector<int64_t> s((size_t)channels * B);
  for (int64_t f0 = 0, fn = 0; f0 < frames; f0 += B, ++fn) {
    const int block = (int)std::min<int64_t>(B, frames - f0);
    for (int c = 0; c < channels; ++c)
      for (int i = 0; i < block; ++i) {
        const float v = in[(f0 + i) * channels + c] * scale;
        int64_t q = std::isfinite(v) ? (int64_t)std::nearbyint(v) : 0;
        s[(size_t)c * B + i] = q < lo ? lo : (q > hi ? hi : q);
      }
    const size_t start = bw.out.size();
    bw.put(0x3FFE, 14);
    bw.put(0, 1);
    bw.put(0, 1);
    bw.put(block == B ? 12 : 7, 4);
    bw.put(rcode, 4);
    bw.put(channels - 1, 4);
    bw.put(bits == 16 ? 4 : 6, 3);
    bw.put(0, 1);
    put_utf8(bw, (uint64_t)fn);
    if (block != B) bw.put(block - 1, 16);
    bw.put(crc8(bw.out.data() + start, bw.out.size() - start), 8);
    for (int c = 0; c < channels; ++c) encode_subframe(bw, s.data() + (size_t)c * B, block, bits);
    bw.align();
    const uint16_t c16 = crc16(bw.out.data() + start, bw.out.size() - start);
    bw.put(c16, 16);
  }
  SESA_REQUIRE(bw.out.size() <= cap, SESA_ERR_INVALID, "flac_encode: output buffer too small (%zu < %zu)", cap,
               bw.out.size());
  memcpy(out, bw.out.data(), bw.out.size());
  *written = bw.out.size();
  return SESA_OK;
}
