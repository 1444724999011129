#include "codec.h"

#include <cstring>
#include <stdexcept>

namespace dryad {

int field_width(FieldKind k) {
  switch (k) {
    case FieldKind::U8: case FieldKind::I8: case FieldKind::Bool: return 1;
    case FieldKind::I16: case FieldKind::U16: return 2;
    case FieldKind::I32: case FieldKind::U32: case FieldKind::F32: return 4;
    case FieldKind::I64: case FieldKind::U64: case FieldKind::F64: case FieldKind::DateTime: return 8;
    case FieldKind::Decimal: case FieldKind::Guid: return 16;
    case FieldKind::String: return 0;
  }
  return 0;
}

size_t read_compact(const uint8_t* p, const uint8_t* end, int32_t* v) {
  if (p >= end) return 0;
  const uint8_t b1 = p[0];
  if (b1 < 0x80) {
    *v = b1;
    return 1;
  }
  if (p + 4 > end) return 0;
  *v = (int32_t)(((uint32_t)(b1 & 0x7F) << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
  return 4;
}

int32_t utf16_units(const uint8_t* s, size_t n) {
  int32_t u = 0;
  for (size_t i = 0; i < n;) {
    const uint8_t c = s[i];
    if (c < 0x80) { i += 1; u += 1; }
    else if (c < 0xE0) { i += 2; u += 1; }
    else if (c < 0xF0) { i += 3; u += 1; }
    else { i += 4; u += 2; }
  }
  return u;
}

size_t decode_records(const uint8_t* buf, size_t len, const std::vector<FieldKind>& schema,
                      std::vector<std::vector<uint8_t>>& fixed, std::vector<StringColumn>& strings) {
  fixed.assign(schema.size(), {});
  strings.assign(schema.size(), {});
  for (size_t f = 0; f < schema.size(); ++f)
    if (schema[f] == FieldKind::String) strings[f].offsets.push_back(0);
  const uint8_t* p = buf;
  const uint8_t* end = buf + len;
  size_t n = 0;
  while (p < end) {
    for (size_t f = 0; f < schema.size(); ++f) {
      const FieldKind k = schema[f];
      if (k == FieldKind::String) {
        int32_t nchars = 0, nbytes = 0;
        size_t c = read_compact(p, end, &nchars);
        if (!c) throw std::runtime_error("truncated record stream (string length)");
        p += c;
        c = read_compact(p, end, &nbytes);
        if (!c) throw std::runtime_error("truncated record stream (string bytes)");
        p += c;
        if (nbytes < 0 || p + nbytes > end) throw std::runtime_error("truncated record stream (string data)");
        StringColumn& sc = strings[f];
        sc.data.insert(sc.data.end(), p, p + nbytes);
        sc.offsets.push_back((int64_t)sc.data.size());
        p += nbytes;
      } else {
        const int w = field_width(k);
        if (p + w > end) throw std::runtime_error("truncated record stream (fixed field)");
        fixed[f].insert(fixed[f].end(), p, p + w);
        p += w;
      }
    }
    ++n;
  }
  return n;
}

size_t scan_record_blocks(const uint8_t* buf, size_t len, const std::vector<FieldKind>& schema, size_t block,
                          std::vector<int64_t>& offsets) {
  if (block == 0) throw std::invalid_argument("scan_record_blocks: block size 0");
  offsets.clear();
  int fixed = 0;
  bool var = false;
  for (FieldKind k : schema) {
    if (k == FieldKind::String) var = true;
    else fixed += field_width(k);
  }
  if (!var) {             // fixed-width records: the offsets are arithmetic
    if (fixed == 0 || len % (size_t)fixed) throw std::runtime_error("record stream length is not a multiple of the record width");
    const size_t n = len / (size_t)fixed;
    for (size_t r = 0; r < n; r += block) offsets.push_back((int64_t)(r * (size_t)fixed));
    return n;
  }
  const uint8_t* p = buf;
  const uint8_t* end = buf + len;
  size_t n = 0;
  while (p < end) {
    if (n % block == 0) offsets.push_back((int64_t)(p - buf));
    for (FieldKind k : schema) {
      if (k == FieldKind::String) {
        int32_t nchars = 0, nbytes = 0;
        size_t c = read_compact(p, end, &nchars);
        if (!c) throw std::runtime_error("truncated record stream (string length)");
        p += c;
        c = read_compact(p, end, &nbytes);
        if (!c) throw std::runtime_error("truncated record stream (string bytes)");
        p += c;
        if (nbytes < 0 || p + nbytes > end) throw std::runtime_error("truncated record stream (string data)");
        p += nbytes;
      } else {
        const int w = field_width(k);
        if (p + w > end) throw std::runtime_error("truncated record stream (fixed field)");
        p += w;
      }
    }
    ++n;
  }
  return n;
}

std::vector<uint8_t> encode_records(size_t n, const std::vector<FieldKind>& schema,
                                    const std::vector<const uint8_t*>& fixed,
                                    const std::vector<const StringColumn*>& strings) {
  size_t est = 0;
  for (size_t f = 0; f < schema.size(); ++f) {
    if (schema[f] == FieldKind::String) est += strings[f]->data.size() + 8 * n;
    else est += (size_t)field_width(schema[f]) * n;
  }
  std::vector<uint8_t> out;
  out.reserve(est);
  uint8_t tmp[8];
  for (size_t i = 0; i < n; ++i) {
    for (size_t f = 0; f < schema.size(); ++f) {
      const FieldKind k = schema[f];
      if (k == FieldKind::String) {
        const StringColumn& sc = *strings[f];
        const int64_t b = sc.offsets[i], e = sc.offsets[i + 1];
        const uint8_t* s = sc.data.data() + b;
        const int32_t nbytes = (int32_t)(e - b);
        const int32_t units = utf16_units(s, (size_t)nbytes);
        size_t c = write_compact(tmp, units);
        out.insert(out.end(), tmp, tmp + c);
        // width of the byte-count field is chosen from the max UTF-8 size (units+1)*3
        const int32_t maxbytes = (units + 1) * 3;
        if (maxbytes < 0x80) {
          out.push_back((uint8_t)nbytes);
        } else {
          tmp[0] = (uint8_t)(((uint32_t)nbytes >> 24) | 0x80);
          tmp[1] = (uint8_t)(nbytes >> 16);
          tmp[2] = (uint8_t)(nbytes >> 8);
          tmp[3] = (uint8_t)nbytes;
          out.insert(out.end(), tmp, tmp + 4);
        }
        out.insert(out.end(), s, s + nbytes);
      } else {
        const int w = field_width(k);
        const uint8_t* src = fixed[f] + (size_t)w * i;
        out.insert(out.end(), src, src + w);
      }
    }
  }
  return out;
}

void split_lines(const uint8_t* buf, size_t len, std::vector<int64_t>& starts, std::vector<int64_t>& ends) {
  size_t i = 0, s = 0;
  while (i < len) {
    const uint8_t c = buf[i];
    if (c == '\n' || c == '\r') {
      starts.push_back((int64_t)s);
      ends.push_back((int64_t)i);
      if (c == '\r' && i + 1 < len && buf[i + 1] == '\n') ++i;
      ++i;
      s = i;
    } else {
      ++i;
    }
  }
  if (s < len) {
    starts.push_back((int64_t)s);
    ends.push_back((int64_t)len);
  }
}

std::vector<uint8_t> lines_to_records(const uint8_t* buf, size_t len) {
  std::vector<int64_t> st, en;
  split_lines(buf, len, st, en);
  StringColumn sc;
  sc.offsets.reserve(st.size() + 1);
  sc.offsets.push_back(0);
  sc.data.reserve(len);
  for (size_t i = 0; i < st.size(); ++i) {
    sc.data.insert(sc.data.end(), buf + st[i], buf + en[i]);
    sc.offsets.push_back((int64_t)sc.data.size());
  }
  std::vector<FieldKind> schema{FieldKind::String};
  std::vector<const uint8_t*> fx{nullptr};
  std::vector<const StringColumn*> ss{&sc};
  return encode_records(st.size(), schema, fx, ss);
}

// ---------------------------------------------------------------------------------------------
// Rabin fingerprints: tab_[b][i] = i * X^(64 + 8b) mod P in the bit-reflected representation
// (the x^63 coefficient is the lsb).  Multiplying by X is a right shift with conditional xor.
Rabin64::Rabin64(uint64_t poly) : poly_(poly) {
  uint64_t f = poly;   // X^64 mod P in this representation
  for (int b = 0; b < 8; ++b) {
    tab_[b][0] = 0;
    for (int i = 0x80; i != 0; i >>= 1) {
      tab_[b][i] = f;
      f = (f >> 1) ^ ((f & 1) ? poly : 0);
    }
    for (int i = 1; i < 256; i <<= 1)
      for (int k = 1; k < i; ++k) tab_[b][i + k] = tab_[b][i] ^ tab_[b][k];
  }
}

uint64_t Rabin64::extend(uint64_t fp, const uint8_t* d, size_t n) const {
  for (size_t i = 0; i < n; ++i) fp = (fp >> 8) ^ tab_[0][(fp & 0xFF) ^ d[i]];
  return fp;
}

uint64_t Rabin64::extend_u16(uint64_t fp, uint16_t v) const {
  fp ^= v;
  return (fp >> 16) ^ tab_[1][fp & 0xFF] ^ tab_[0][(fp >> 8) & 0xFF];
}

uint64_t Rabin64::extend_u32(uint64_t fp, uint32_t v) const {
  fp ^= v;
  return (fp >> 32) ^ tab_[3][fp & 0xFF] ^ tab_[2][(fp >> 8) & 0xFF] ^ tab_[1][(fp >> 16) & 0xFF] ^
         tab_[0][(fp >> 24) & 0xFF];
}

uint64_t Rabin64::extend_u64(uint64_t fp, uint64_t v) const {
  fp ^= v;
  uint64_t r = 0;
  for (int b = 0; b < 8; ++b) r ^= tab_[7 - b][(fp >> (8 * b)) & 0xFF];
  return r;
}

}  // namespace dryad
