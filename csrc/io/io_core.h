// hopsx IO core: the parsers and codecs of _hopsx_io without any Python types, so the same code
// runs in the extension (io.cpp) and in the native AddressSanitizer / UBSan fuzz harness
// (tools/asan/io_fuzz.cpp, tests/test_io_asan.py).
//
// Every parser takes untrusted bytes (files a user points a reader at): lengths read from the
// input are checked against the bytes that remain BEFORE any pointer moves or copy happens, with
// overflow-safe arithmetic, and malformed input raises std::runtime_error — it never reads past
// the buffer.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#if defined(__SSE4_2__)
#include <nmmintrin.h>
#endif

namespace hopsx_io {

// ------------------------------------------------------------------ crc32c
inline uint32_t crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
#if defined(__SSE4_2__)
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c64 = _mm_crc32_u64(c64, v);
    p += 8;
    n -= 8;
  }
  c = (uint32_t)c64;
  while (n--) c = _mm_crc32_u8(c, *p++);
#else
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t t = i;
      for (int k = 0; k < 8; ++k) t = (t & 1) ? (t >> 1) ^ 0x82F63B78u : (t >> 1);
      table[i] = t;
    }
    init = true;
  }
  while (n--) c = table[(c ^ *p++) & 0xFF] ^ (c >> 8);
#endif
  return c ^ 0xFFFFFFFFu;
}

inline uint32_t masked_crc(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ---------------------------------------------------------------- TFRecord
// frame = u64 length | u32 masked crc(length) | payload | u32 masked crc(payload)
inline std::string frame_record(const uint8_t* d, size_t n) {
  std::string o(12 + n + 4, '\0');
  const uint64_t len = n;
  memcpy(&o[0], &len, 8);
  const uint32_t lc = masked_crc((const uint8_t*)o.data(), 8);
  memcpy(&o[8], &lc, 4);
  if (n) memcpy(&o[12], d, n);
  const uint32_t dc = masked_crc(d, n);
  memcpy(&o[12 + n], &dc, 4);
  return o;
}

// (offset, length) of every payload; the length field is bounds-checked against the remaining
// bytes before it is used (a corrupt 64-bit length cannot wrap the check)
inline std::vector<std::pair<size_t, size_t>> index_records(const uint8_t* b, size_t size, bool verify) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t pos = 0;
  while (size - pos >= 12) {
    uint64_t len;
    memcpy(&len, b + pos, 8);
    if (verify) {
      uint32_t lc;
      memcpy(&lc, b + pos + 8, 4);
      if (lc != masked_crc(b + pos, 8)) throw std::runtime_error("TFRecord length crc mismatch");
    }
    const size_t rest = size - pos - 12;
    if (rest < 4 || len > rest - 4) throw std::runtime_error("truncated TFRecord");
    if (verify) {
      uint32_t dc;
      memcpy(&dc, b + pos + 12 + len, 4);
      if (dc != masked_crc(b + pos + 12, len)) throw std::runtime_error("TFRecord data crc mismatch");
    }
    out.emplace_back(pos + 12, (size_t)len);
    pos += 12 + len + 4;
  }
  if (pos != size) throw std::runtime_error("trailing bytes after the last TFRecord");
  return out;
}

// ------------------------------------------------------- protobuf helpers
inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
inline void put_key(std::string& o, int field, int wire) { put_varint(o, ((uint64_t)field << 3) | wire); }
inline void put_len(std::string& o, int field, const std::string& s) {
  put_key(o, field, 2);
  put_varint(o, s.size());
  o += s;
}

inline uint64_t get_varint(const uint8_t*& p, const uint8_t* end) {
  uint64_t v = 0;
  for (int sh = 0; p < end && sh < 64; sh += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) return v;
  }
  throw std::runtime_error("malformed varint");
}

// a length-delimited field's length, checked against the bytes left
inline size_t get_len(const uint8_t*& p, const uint8_t* end) {
  const uint64_t n = get_varint(p, end);
  if (n > (uint64_t)(end - p)) throw std::runtime_error("length-delimited field runs past its message");
  return (size_t)n;
}

inline void advance(const uint8_t*& p, const uint8_t* end, size_t n) {
  if (n > (size_t)(end - p)) throw std::runtime_error("field runs past its message");
  p += n;
}

inline void skip_field(const uint8_t*& p, const uint8_t* end, int wire) {
  if (wire == 0) get_varint(p, end);
  else if (wire == 1) advance(p, end, 8);
  else if (wire == 2) advance(p, end, get_len(p, end));
  else if (wire == 5) advance(p, end, 4);
  else throw std::runtime_error("unsupported wire type");
}

struct FeatVal {
  int kind = -1;  // 0 bytes, 1 float, 2 int64
  std::vector<float> f;
  std::vector<int64_t> i;
  std::vector<std::string> b;
};

inline void parse_list(const uint8_t* p, const uint8_t* end, int kind, FeatVal& fv) {
  fv.kind = kind;
  while (p < end) {
    const uint64_t key = get_varint(p, end);
    const int field = (int)(key >> 3), wire = (int)(key & 7);
    if (field != 1) {
      skip_field(p, end, wire);
      continue;
    }
    if (kind == 0) {
      if (wire != 2) throw std::runtime_error("BytesList value is not length-delimited");
      const size_t n = get_len(p, end);
      fv.b.emplace_back((const char*)p, n);
      p += n;
    } else if (kind == 1) {
      if (wire == 2) {
        const size_t n = get_len(p, end);
        if (n % 4) throw std::runtime_error("packed FloatList length is not a multiple of 4");
        const size_t off = fv.f.size();
        fv.f.resize(off + n / 4);
        if (n) memcpy(fv.f.data() + off, p, n);
        p += n;
      } else if (wire == 5) {
        float v;
        if (end - p < 4) throw std::runtime_error("truncated float");
        memcpy(&v, p, 4);
        p += 4;
        fv.f.push_back(v);
      } else {
        throw std::runtime_error("FloatList value has a bad wire type");
      }
    } else {
      if (wire == 2) {
        const size_t n = get_len(p, end);
        const uint8_t* e = p + n;
        while (p < e) fv.i.push_back((int64_t)get_varint(p, e));
      } else if (wire == 0) {
        fv.i.push_back((int64_t)get_varint(p, end));
      } else {
        throw std::runtime_error("Int64List value has a bad wire type");
      }
    }
  }
}

// tf.train.Example: Example{1: Features{1: map<string, Feature>}}; Feature oneof
// {1: BytesList{1: repeated bytes}, 2: FloatList{1: packed float}, 3: Int64List{1: packed int64}}
inline std::unordered_map<std::string, FeatVal> parse_example(const uint8_t* p, const uint8_t* end) {
  std::unordered_map<std::string, FeatVal> out;
  while (p < end) {
    const uint64_t key = get_varint(p, end);
    if ((key >> 3) != 1 || (key & 7) != 2) {
      skip_field(p, end, key & 7);
      continue;
    }
    const size_t flen = get_len(p, end);  // (a separate statement: get_len advances p)
    const uint8_t* fe = p + flen;
    while (p < fe) {  // Features: repeated map entries (field 1)
      const uint64_t k2 = get_varint(p, fe);
      if ((k2 & 7) != 2) {
        skip_field(p, fe, k2 & 7);
        continue;
      }
      const size_t elen = get_len(p, fe);
      const uint8_t* ee = p + elen;
      if ((k2 >> 3) != 1) {
        p = ee;
        continue;
      }
      std::string name;
      FeatVal fv;
      while (p < ee) {
        const uint64_t k3 = get_varint(p, ee);
        if ((k3 & 7) != 2) {
          skip_field(p, ee, k3 & 7);
          continue;
        }
        const size_t l3 = get_len(p, ee);
        if ((k3 >> 3) == 1) {
          name.assign((const char*)p, l3);
          p += l3;
        } else if ((k3 >> 3) == 2) {
          const uint8_t* fe2 = p + l3;
          while (p < fe2) {  // Feature oneof
            const uint64_t k4 = get_varint(p, fe2);
            if ((k4 & 7) != 2) {
              skip_field(p, fe2, k4 & 7);
              continue;
            }
            const size_t l4 = get_len(p, fe2);
            const int which = (int)(k4 >> 3);
            if (which >= 1 && which <= 3) parse_list(p, p + l4, which == 1 ? 0 : (which == 2 ? 1 : 2), fv);
            p += l4;
          }
        } else {
          p += l3;
        }
      }
      out[std::move(name)] = std::move(fv);
    }
  }
  return out;
}

// ---------------------------------------------------------------- CSV
struct CsvTable {
  std::vector<std::string> names;
  std::vector<float> vals;  // row-major [nrows][ncols]; empty / non-numeric fields are NaN
  size_t nrows = 0, ncols = 0;
};

inline CsvTable parse_csv_numeric(const char* buf, size_t size, char delim, bool header) {
  CsvTable t;
  size_t pos = 0;
  auto next_line = [&](size_t& s, size_t& e) -> bool {
    if (pos >= size) return false;
    s = pos;
    const void* nl = memchr(buf + pos, '\n', size - pos);
    e = nl ? (size_t)((const char*)nl - buf) : size;
    pos = e + 1;
    if (e > s && buf[e - 1] == '\r') --e;
    return true;
  };
  size_t s, e;
  if (header && next_line(s, e)) {
    std::string cur;
    bool q = false;
    for (size_t i = s; i < e; ++i) {
      const char c = buf[i];
      if (c == '"') q = !q;
      else if (c == delim && !q) {
        t.names.push_back(cur);
        cur.clear();
      } else {
        cur.push_back(c);
      }
    }
    t.names.push_back(cur);
  }
  t.ncols = t.names.size();
  std::string field;
  while (next_line(s, e)) {
    if (e == s) continue;
    size_t col = 0, fs = s;
    bool q = false;
    for (size_t i = s; i <= e; ++i) {
      const bool last = (i == e);
      if (!last && buf[i] == '"') q = !q;
      if (last || (buf[i] == delim && !q)) {
        field.assign(buf + fs, i - fs);
        if (field.size() >= 2 && field.front() == '"' && field.back() == '"') field = field.substr(1, field.size() - 2);
        float v = NAN;
        if (!field.empty()) {
          char* ep = nullptr;
          v = strtof(field.c_str(), &ep);
          while (ep && *ep == ' ') ++ep;
          if (!ep || *ep != '\0') v = NAN;
        }
        t.vals.push_back(v);
        ++col;
        fs = i + 1;
      }
    }
    if (t.ncols == 0) t.ncols = col;
    if (col < t.ncols)
      for (; col < t.ncols; ++col) t.vals.push_back(NAN);
    else if (col > t.ncols)
      t.vals.resize(t.vals.size() - (col - t.ncols));
    ++t.nrows;
  }
  return t;
}

}  // namespace hopsx_io
