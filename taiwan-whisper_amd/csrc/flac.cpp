// FLAC decoder (host code): the reference reads its NTU-COOL corpus with soundfile / libsndfile
// (dataset/cool_dataset.py:55, `sf.read(path)` of `.flac`), which this image lacks; this restates the
// format (RFC 9639: STREAMINFO, frame header with CRC-8, CONSTANT / VERBATIM / FIXED / LPC subframes,
// wasted bits, Rice-coded residuals with escape partitions, independent / left-side / side-right /
// mid-side channels, CRC-16 frame footer) so tw.dataset.read_audio decodes `.flac` natively.
//
//   tw_flac_info(data, n, info)                 info = {channels, sample_rate, bits_per_sample,
//                                                       total samples per channel (0 = unknown)}
//   tw_flac_decode(data, n, out, cap, &frames)  interleaved int32 samples, `frames` per channel decoded
//
// Status: 0 ok, TW_EINVAL malformed stream (bad marker / sync / CRC / reserved codes), TW_EUNSUPPORTED
// a valid stream outside what the reference's corpus needs (> 8 channels cannot occur; none today).
#include <cstdint>
#include <cstring>
#include <vector>

#include "tw_hip.h"

namespace {

constexpr int TW_OK = 0, TW_EINVAL = 1, TW_EUNSUPPORTED = 2;

constexpr int OK = 0, EINV = 1, EUNS = 2;

struct Bits {
  const uint8_t* p;
  int64_t n;        // bytes
  int64_t pos = 0;  // bit position
  bool bad = false;
  uint64_t read(int k) {           // k <= 57
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) {
      if ((pos >> 3) >= n) { bad = true; return 0; }
      v = (v << 1) | ((p[pos >> 3] >> (7 - (pos & 7))) & 1u);
      ++pos;
    }
    return v;
  }
  int64_t read_signed(int k) {
    if (k == 0) return 0;
    const uint64_t v = read(k);
    return (int64_t)(v << (64 - k)) >> (64 - k);
  }
  uint32_t unary() {               // zeros before the next 1
    uint32_t q = 0;
    while (true) {
      if ((pos >> 3) >= n) { bad = true; return 0; }
      if ((p[pos >> 3] >> (7 - (pos & 7))) & 1u) { ++pos; return q; }
      ++pos;
      ++q;
    }
  }
  void align() { pos = (pos + 7) & ~int64_t(7); }
};

uint8_t crc8(const uint8_t* d, int64_t n) {       // poly x^8 + x^2 + x + 1
  uint8_t c = 0;
  for (int64_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int b = 0; b < 8; ++b) c = (c & 0x80) ? (uint8_t)((c << 1) ^ 0x07) : (uint8_t)(c << 1);
  }
  return c;
}

uint16_t crc16(const uint8_t* d, int64_t n) {     // poly x^16 + x^15 + x^2 + 1
  uint16_t c = 0;
  for (int64_t i = 0; i < n; ++i) {
    c ^= (uint16_t)d[i] << 8;
    for (int b = 0; b < 8; ++b) c = (c & 0x8000) ? (uint16_t)((c << 1) ^ 0x8005) : (uint16_t)(c << 1);
  }
  return c;
}

struct StreamInfo {
  int channels = 0, rate = 0, bps = 0;
  uint64_t total = 0;
  int64_t first_frame = 0;   // byte offset of the first frame
};

int parse_header(const uint8_t* d, int64_t n, StreamInfo& si) {
  int64_t o = 0;
  if (n >= 10 && d[0] == 'I' && d[1] == 'D' && d[2] == '3') {     // ID3v2 tag in front (skipped)
    const int64_t sz = ((int64_t)(d[6] & 0x7f) << 21) | ((d[7] & 0x7f) << 14) | ((d[8] & 0x7f) << 7) | (d[9] & 0x7f);
    o = 10 + sz;
  }
  if (n < o + 4 || memcmp(d + o, "fLaC", 4) != 0) return EINV;
  o += 4;
  bool have_si = false, last = false;
  while (!last) {
    if (o + 4 > n) return EINV;
    last = d[o] & 0x80;
    const int type = d[o] & 0x7f;
    const int64_t len = ((int64_t)d[o + 1] << 16) | (d[o + 2] << 8) | d[o + 3];
    o += 4;
    if (o + len > n || type == 127) return EINV;
    if (type == 0) {
      if (len < 34) return EINV;
      Bits b{d + o, len};
      b.read(16); b.read(16); b.read(24); b.read(24);
      si.rate = (int)b.read(20);
      si.channels = (int)b.read(3) + 1;
      si.bps = (int)b.read(5) + 1;
      si.total = b.read(36);
      have_si = true;
    }
    o += len;
  }
  if (!have_si || si.bps < 4) return EINV;
  si.first_frame = o;
  return OK;
}

// residual of one subframe into res[pred_order..bs)
int read_residual(Bits& b, int bs, int order, int64_t* out) {
  const int method = (int)b.read(2);
  if (method > 1) return EINV;
  const int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  const int porder = (int)b.read(4);
  const int parts = 1 << porder;
  if ((bs >> porder) < order || (bs & (parts - 1))) return EINV;
  int i = order;
  for (int pt = 0; pt < parts; ++pt) {
    const int cnt = (bs >> porder) - (pt == 0 ? order : 0);
    const int k = (int)b.read(pbits);
    if (k == esc) {
      const int raw = (int)b.read(5);
      for (int j = 0; j < cnt; ++j) out[i++] = b.read_signed(raw);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = b.unary();
        const uint64_t v = (q << k) | b.read(k);
        out[i++] = (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
      }
    }
    if (b.bad) return EINV;
  }
  return OK;
}

int read_subframe(Bits& b, int bs, int bps, int64_t* s) {
  if (b.read(1) != 0) return EINV;
  const int type = (int)b.read(6);
  int wasted = 0;
  if (b.read(1)) wasted = (int)b.unary() + 1;
  if (wasted >= bps) return EINV;
  const int w = bps - wasted;
  if (type == 0) {                                   // CONSTANT
    const int64_t v = b.read_signed(w);
    for (int i = 0; i < bs; ++i) s[i] = v;
  } else if (type == 1) {                            // VERBATIM
    for (int i = 0; i < bs; ++i) s[i] = b.read_signed(w);
  } else if (type >= 8 && type <= 12) {              // FIXED, order 0..4
    const int order = type - 8;
    if (order > bs) return EINV;
    for (int i = 0; i < order; ++i) s[i] = b.read_signed(w);
    if (read_residual(b, bs, order, s) != OK) return EINV;
    for (int i = order; i < bs; ++i) {
      int64_t p = 0;
      switch (order) {
        case 1: p = s[i - 1]; break;
        case 2: p = 2 * s[i - 1] - s[i - 2]; break;
        case 3: p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
        case 4: p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
        default: p = 0;
      }
      s[i] += p;
    }
  } else if (type >= 32) {                           // LPC, order 1..32
    const int order = type - 31;
    if (order > bs) return EINV;
    for (int i = 0; i < order; ++i) s[i] = b.read_signed(w);
    const int prec = (int)b.read(4) + 1;
    if (prec == 16) return EINV;
    const int shift = (int)b.read_signed(5);
    if (shift < 0) return EINV;
    int64_t coef[32];
    for (int j = 0; j < order; ++j) coef[j] = b.read_signed(prec);
    if (read_residual(b, bs, order, s) != OK) return EINV;
    for (int i = order; i < bs; ++i) {
      int64_t acc = 0;
      for (int j = 0; j < order; ++j) acc += coef[j] * s[i - 1 - j];
      s[i] += acc >> shift;
    }
  } else {
    return EINV;                                     // reserved subframe types
  }
  if (b.bad) return EINV;
  if (wasted)
    for (int i = 0; i < bs; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return OK;
}

// Decode every frame.  out == nullptr: count only.  Returns status; *frames = samples per channel.
int decode(const uint8_t* d, int64_t n, const StreamInfo& si, int32_t* out, int64_t cap, int64_t* frames) {
  int64_t o = si.first_frame, done = 0;
  std::vector<int64_t> ch[8];
  while (o + 2 <= n) {
    if (d[o] != 0xff || (d[o + 1] & 0xfe) != 0xf8) {
      if (d[o] == 0) { ++o; continue; }   // trailing padding
      return EINV;
    }
    Bits b{d + o, n - o};
    b.read(15);
    b.read(1);                                       // blocking strategy (fixed / variable)
    const int bs_code = (int)b.read(4), sr_code = (int)b.read(4), ch_code = (int)b.read(4), ss_code = (int)b.read(3);
    if (b.read(1) != 0) return EINV;
    // coded frame / sample number (UTF-8-like, up to 7 bytes)
    const uint64_t first = b.read(8);
    int extra = 0;
    if (first & 0x80) {
      if ((first & 0xe0) == 0xc0) extra = 1;
      else if ((first & 0xf0) == 0xe0) extra = 2;
      else if ((first & 0xf8) == 0xf0) extra = 3;
      else if ((first & 0xfc) == 0xf8) extra = 4;
      else if ((first & 0xfe) == 0xfc) extra = 5;
      else if (first == 0xfe) extra = 6;
      else return EINV;
    }
    for (int i = 0; i < extra; ++i)
      if ((b.read(8) & 0xc0) != 0x80) return EINV;
    int bs = 0;
    if (bs_code == 0) return EINV;
    else if (bs_code == 1) bs = 192;
    else if (bs_code <= 5) bs = 576 << (bs_code - 2);
    else if (bs_code == 6) bs = (int)b.read(8) + 1;
    else if (bs_code == 7) bs = (int)b.read(16) + 1;
    else bs = 256 << (bs_code - 8);
    if (sr_code == 12) b.read(8);
    else if (sr_code == 13 || sr_code == 14) b.read(16);
    else if (sr_code == 15) return EINV;
    int bps = 0;
    switch (ss_code) {
      case 0: bps = si.bps; break;
      case 1: bps = 8; break;
      case 2: bps = 12; break;
      case 4: bps = 16; break;
      case 5: bps = 20; break;
      case 6: bps = 24; break;
      case 7: bps = 32; break;
      default: return EINV;
    }
    if (b.bad) return EINV;
    const int64_t hdr_bytes = b.pos >> 3;
    if (o + hdr_bytes + 1 > n || crc8(d + o, hdr_bytes) != d[o + hdr_bytes]) return EINV;
    b.pos += 8;
    int nch;
    if (ch_code <= 7) nch = ch_code + 1;
    else if (ch_code <= 10) nch = 2;
    else return EINV;
    if (nch != si.channels) return EINV;
    for (int c = 0; c < nch; ++c) {
      ch[c].assign(bs, 0);
      int cb = bps;
      if ((ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1)) cb = bps + 1;  // side
      if (read_subframe(b, bs, cb, ch[c].data()) != OK) return EINV;
    }
    b.align();
    const int64_t body = b.pos >> 3;
    if (o + body + 2 > n) return EINV;
    const uint16_t want = (uint16_t)((d[o + body] << 8) | d[o + body + 1]);
    if (crc16(d + o, body) != want) return EINV;
    if (ch_code == 8) {                               // left / side
      for (int i = 0; i < bs; ++i) ch[1][i] = ch[0][i] - ch[1][i];
    } else if (ch_code == 9) {                        // side / right
      for (int i = 0; i < bs; ++i) ch[0][i] = ch[0][i] + ch[1][i];
    } else if (ch_code == 10) {                       // mid / side
      for (int i = 0; i < bs; ++i) {
        const int64_t side = ch[1][i];
        const int64_t mid = (int64_t)((uint64_t)ch[0][i] << 1) | (side & 1);
        ch[0][i] = (mid + side) >> 1;
        ch[1][i] = (mid - side) >> 1;
      }
    }
    if (out) {
      if ((done + bs) * nch > cap) return EINV;
      for (int i = 0; i < bs; ++i)
        for (int c = 0; c < nch; ++c) out[(done + i) * nch + c] = (int32_t)ch[c][i];
    }
    done += bs;
    o += body + 2;
  }
  *frames = done;
  return OK;
}

}  // namespace

extern "C" int tw_flac_info(const uint8_t* data, int64_t n, int64_t* info) {
  if (!data || n <= 0 || !info) return TW_EINVAL;
  StreamInfo si;
  const int st = parse_header(data, n, si);
  if (st != OK) return TW_EINVAL;
  info[0] = si.channels;
  info[1] = si.rate;
  info[2] = si.bps;
  info[3] = (int64_t)si.total;
  return TW_OK;
}

extern "C" int tw_flac_decode(const uint8_t* data, int64_t n, int32_t* out, int64_t cap, int64_t* frames) {
  if (!data || n <= 0 || !frames) return TW_EINVAL;
  StreamInfo si;
  if (parse_header(data, n, si) != OK) return TW_EINVAL;
  const int st = decode(data, n, si, out, cap, frames);
  return st == OK ? TW_OK : (st == EUNS ? TW_EUNSUPPORTED : TW_EINVAL);
}
