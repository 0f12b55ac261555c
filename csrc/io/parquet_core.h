// hopsx native Parquet column decoder: footer (Thrift compact protocol) -> row-group / column-chunk
// plan -> page decode (PLAIN, dictionary, RLE/bit-packed definition levels, UNCOMPRESSED or SNAPPY)
// straight into a caller-owned buffer — the pinned staging ring of the Parquet -> HBM reader
// (hops_examples_amd/io/parquet.py).  No Arrow, no Python objects, no intermediate copies: the
// values of one column chunk land at their final offset in the staging slot that the next H2D copy
// sends to the GPU, where one kernel converts + interleaves every column (columns.hip).
//
// Scope: flat schemas of BOOLEAN / INT32 / INT64 / FLOAT / DOUBLE columns (REQUIRED or OPTIONAL:
// nulls are filled with NaN for floating columns, 0 otherwise), data pages v1 and v2, dictionary
// pages; codecs NONE and SNAPPY.  Anything else throws hopsx_io::Unsupported and the reader falls
// back to Arrow for that file.  Inputs are untrusted (the file a user points a reader at): every
// length read from the file is checked against the bytes that remain before it is used.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace hopsx_io {

struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ Thrift compact protocol
class Thrift {
 public:
  Thrift(const uint8_t* p, size_t n) : p_(p), end_(p + n) {}
  size_t pos(const uint8_t* base) const { return (size_t)(p_ - base); }
  const uint8_t* cur() const { return p_; }

  uint8_t byte() {
    need(1);
    return *p_++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      const uint8_t b = byte();
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("parquet: varint too long");
  }
  int64_t zigzag() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  std::string binary() {
    const uint64_t n = varint();
    need(n);
    std::string s((const char*)p_, (size_t)n);
    p_ += n;
    return s;
  }
  // field header: returns (id, type); type 0 = stop.  `last` carries the previous id of the struct.
  bool field(int& id, int& type, int& last) {
    const uint8_t h = byte();
    if (h == 0) return false;
    type = h & 0x0F;
    const int delta = h >> 4;
    id = delta ? last + delta : (int)(int16_t)zigzag();
    last = id;
    return true;
  }
  // list / set header: (size, element type)
  void list(uint64_t& n, int& et) {
    const uint8_t h = byte();
    et = h & 0x0F;
    n = h >> 4;
    if (n == 15) n = varint();
    if (n > (uint64_t)(end_ - p_) + 1) throw std::runtime_error("parquet: list size exceeds the footer");
  }
  void skip(int type, int depth = 0) {
    if (depth > 32) throw std::runtime_error("parquet: thrift nesting too deep");
    switch (type) {
      case 1:  // bool true
      case 2:  // bool false
        return;
      case 3:
        byte();
        return;
      case 4:
      case 5:
      case 6:
        varint();
        return;
      case 7:
        need(8);
        p_ += 8;
        return;
      case 8: {
        const uint64_t n = varint();
        need(n);
        p_ += n;
        return;
      }
      case 9:
      case 10: {
        uint64_t n;
        int et;
        list(n, et);
        for (uint64_t i = 0; i < n; ++i) skip(et == 1 || et == 2 ? 3 : et, depth + 1);  // list bools are bytes
        return;
      }
      case 11: {
        const uint64_t n = varint();
        if (!n) return;
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n; ++i) {
          skip(kv >> 4, depth + 1);
          skip(kv & 0x0F, depth + 1);
        }
        return;
      }
      case 12: {
        int id, t, last = 0;
        while (field(id, t, last)) skip(t, depth + 1);
        return;
      }
      default:
        throw std::runtime_error("parquet: bad thrift type");
    }
  }

 private:
  void need(uint64_t n) const {
    if (n > (uint64_t)(end_ - p_)) throw std::runtime_error("parquet: truncated thrift structure");
  }
  const uint8_t* p_;
  const uint8_t* end_;
};

// ------------------------------------------------------------------ file metadata
enum PType : int { PT_BOOLEAN = 0, PT_INT32 = 1, PT_INT64 = 2, PT_INT96 = 3, PT_FLOAT = 4, PT_DOUBLE = 5,
                   PT_BYTE_ARRAY = 6, PT_FIXED = 7 };

struct PqColumn {  // a leaf of a flat schema
  std::string name;
  int type = -1;
  int repetition = 0;  // 0 required, 1 optional, 2 repeated
  // false when a converted type / logical type changes what the physical values mean (DECIMAL scale,
  // unsigned, DATE/TIME/TIMESTAMP units, strings...): the raw values are then not the column's values,
  // and the reader must take the Arrow path.  Plain: no annotation, or a signed INT_8..INT_64.
  bool plain = true;
};
struct PqChunk {
  int type = -1, codec = 0;
  int64_t num_values = 0, data_page_offset = -1, dict_page_offset = -1, total_compressed = 0;
};
struct PqRowGroup {
  int64_t num_rows = 0;
  std::vector<PqChunk> chunks;
};
struct PqMeta {
  std::vector<PqColumn> columns;
  std::vector<PqRowGroup> row_groups;
  int64_t num_rows = 0;
};

inline int ptype_width(int t) {
  switch (t) {
    case PT_BOOLEAN: return 1;  // one byte per value in the output
    case PT_INT32: case PT_FLOAT: return 4;
    case PT_INT64: case PT_DOUBLE: return 8;
    default: return 0;
  }
}

inline PqChunk parse_column_meta(Thrift& t) {
  PqChunk c;
  int id, ty, last = 0;
  while (t.field(id, ty, last)) {
    if (id == 1 && ty == 5) c.type = (int)t.zigzag();
    else if (id == 4 && ty == 5) c.codec = (int)t.zigzag();
    else if (id == 5 && ty == 6) c.num_values = t.zigzag();
    else if (id == 7 && ty == 6) c.total_compressed = t.zigzag();
    else if (id == 9 && ty == 6) c.data_page_offset = t.zigzag();
    else if (id == 11 && ty == 6) c.dict_page_offset = t.zigzag();
    else t.skip(ty);
  }
  return c;
}

inline PqMeta parse_footer(const uint8_t* data, size_t size) {
  if (size < 12 || std::memcmp(data, "PAR1", 4) || std::memcmp(data + size - 4, "PAR1", 4))
    throw std::runtime_error("parquet: not a Parquet file (magic)");
  uint32_t flen;
  std::memcpy(&flen, data + size - 8, 4);
  if ((uint64_t)flen + 12 > size) throw std::runtime_error("parquet: footer length exceeds the file");
  Thrift t(data + size - 8 - flen, flen);
  PqMeta m;
  std::vector<PqColumn> schema;
  int id, ty, last = 0;
  while (t.field(id, ty, last)) {
    if (id == 2 && ty == 9) {
      uint64_t n;
      int et;
      t.list(n, et);
      for (uint64_t i = 0; i < n; ++i) {
        PqColumn c;
        int nchild = 0;
        int fid, fty, flast = 0;
        while (t.field(fid, fty, flast)) {
          if (fid == 1 && fty == 5) c.type = (int)t.zigzag();
          else if (fid == 3 && fty == 5) c.repetition = (int)t.zigzag();
          else if (fid == 4 && fty == 8) c.name = t.binary();
          else if (fid == 5 && fty == 5) nchild = (int)t.zigzag();
          else if (fid == 6 && fty == 5) {  // converted_type: INT_8..INT_64 (15..18) keep plain values
            const int64_t ct = t.zigzag();
            if (ct < 15 || ct > 18) c.plain = false;
          } else if (fid == 7 && fty == 5) {  // scale (DECIMAL)
            if (t.zigzag() != 0) c.plain = false;
          } else if (fid == 10 && fty == 12) {  // logicalType union: only a signed INTEGER stays plain
            int lid, lty, llast = 0;
            while (t.field(lid, lty, llast)) {
              if (lid == 10 && lty == 12) {  // IntType {1: bitWidth i8, 2: isSigned bool}
                int iid, ity, ilast = 0;
                while (t.field(iid, ity, ilast)) {
                  if (iid == 2 && (ity == 1 || ity == 2)) {
                    if (ity == 2) c.plain = false;  // compact-protocol bool false
                  } else {
                    t.skip(ity);
                  }
                }
              } else {
                c.plain = false;
                t.skip(lty);
              }
            }
          } else {
            t.skip(fty);
          }
        }
        if (i == 0) continue;  // the root
        if (nchild > 0) throw Unsupported("parquet: nested schema");
        schema.push_back(c);
      }
    } else if (id == 3 && ty == 6) {
      m.num_rows = t.zigzag();
    } else if (id == 4 && ty == 9) {
      uint64_t n;
      int et;
      t.list(n, et);
      for (uint64_t i = 0; i < n; ++i) {
        PqRowGroup rg;
        int rid, rty, rlast = 0;
        while (t.field(rid, rty, rlast)) {
          if (rid == 1 && rty == 9) {
            uint64_t nc;
            int cet;
            t.list(nc, cet);
            for (uint64_t j = 0; j < nc; ++j) {
              PqChunk ch;
              int cid, cty, clast = 0;
              while (t.field(cid, cty, clast)) {
                if (cid == 1 && cty == 8) {
                  if (!t.binary().empty()) throw Unsupported("parquet: column chunk in another file");
                } else if (cid == 3 && cty == 12) {
                  ch = parse_column_meta(t);
                } else {
                  t.skip(cty);
                }
              }
              rg.chunks.push_back(ch);
            }
          } else if (rid == 3 && rty == 6) {
            rg.num_rows = t.zigzag();
          } else {
            t.skip(rty);
          }
        }
        m.row_groups.push_back(std::move(rg));
      }
    } else {
      t.skip(ty);
    }
  }
  m.columns = std::move(schema);
  for (auto& rg : m.row_groups)
    if (rg.chunks.size() != m.columns.size()) throw std::runtime_error("parquet: row group / schema mismatch");
  return m;
}

// ------------------------------------------------------------------ snappy (raw block format)
inline void snappy_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t expect) {
  Thrift v(src, n);  // varint reader
  const uint64_t len = v.varint();
  if (len != expect) throw std::runtime_error("parquet: snappy length mismatch");
  out.resize((size_t)len);
  size_t ip = v.pos(src), op = 0;
  while (ip < n) {
    const uint8_t tag = src[ip++];
    const int kind = tag & 3;
    if (kind == 0) {  // literal
      size_t l = tag >> 2;
      if (l >= 60) {
        const int nb = (int)l - 59;
        if (ip + nb > n) throw std::runtime_error("parquet: snappy literal truncated");
        l = 0;
        for (int i = 0; i < nb; ++i) l |= (size_t)src[ip + i] << (8 * i);
        ip += nb;
      }
      l += 1;
      if (l > n - ip || l > len - op) throw std::runtime_error("parquet: snappy literal out of range");
      std::memcpy(out.data() + op, src + ip, l);
      ip += l;
      op += l;
    } else {
      size_t l, off;
      if (kind == 1) {
        if (ip + 1 > n) throw std::runtime_error("parquet: snappy copy truncated");
        l = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | src[ip];
        ip += 1;
      } else if (kind == 2) {
        if (ip + 2 > n) throw std::runtime_error("parquet: snappy copy truncated");
        l = 1 + (tag >> 2);
        off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) throw std::runtime_error("parquet: snappy copy truncated");
        l = 1 + (tag >> 2);
        off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8) | ((size_t)src[ip + 2] << 16) |
              ((size_t)src[ip + 3] << 24);
        ip += 4;
      }
      if (off == 0 || off > op || l > len - op) throw std::runtime_error("parquet: snappy copy out of range");
      uint8_t* d = out.data() + op;
      const uint8_t* s = d - off;
      size_t i = 0;
      if (off >= 8)  // 8-byte chunks never read bytes this copy writes
        for (; i + 8 <= l; i += 8) std::memcpy(d + i, s + i, 8);
      for (; i < l; ++i) d[i] = s[i];  // (offsets < 8: overlapping forward run-length copies, byte-wise)
      op += l;
    }
  }
  if (op != len) throw std::runtime_error("parquet: snappy output short");
}

// ------------------------------------------------------------------ RLE / bit-packed hybrid
// Decodes `count` values of `bw` bits from p[0, n); returns the bytes consumed.
inline size_t rle_hybrid(const uint8_t* p, size_t n, int bw, uint32_t* outv, size_t count) {
  if (bw < 0 || bw > 32) throw std::runtime_error("parquet: bad bit width");
  size_t ip = 0, got = 0;
  const size_t vb = (size_t)(bw + 7) / 8;
  const uint64_t mask = bw == 32 ? 0xFFFFFFFFull : ((1ull << bw) - 1);
  while (got < count) {
    if (ip >= n) throw std::runtime_error("parquet: levels / indices truncated");
    Thrift t(p + ip, n - ip);
    const uint64_t h = t.varint();
    ip += t.pos(p + ip);
    if (!(h & 1)) {  // RLE run: (h >> 1) copies of one little-endian value of vb bytes
      if (vb > n - ip) throw std::runtime_error("parquet: rle value truncated");
      uint32_t v = 0;
      for (size_t i = 0; i < vb; ++i) v |= (uint32_t)p[ip + i] << (8 * i);
      ip += vb;
      const size_t m = (size_t)std::min<uint64_t>(h >> 1, count - got);
      for (size_t i = 0; i < m; ++i) outv[got + i] = v;
      got += m;
    } else {  // (h >> 1) bit-packed groups of 8 values, LSB first
      const uint64_t groups = h >> 1;
      if (groups > (n - ip) / (bw ? (uint64_t)bw : 1ull) + 1) throw std::runtime_error("parquet: bit-packed run truncated");
      const uint64_t nbytes = groups * (uint64_t)bw;
      if (nbytes > n - ip) throw std::runtime_error("parquet: bit-packed run truncated");
      const uint8_t* q = p + ip;
      for (uint64_t i = 0; i < groups * 8 && got < count; ++i, ++got) {
        const uint64_t bit = i * (uint64_t)bw;
        const uint64_t b0 = bit >> 3;
        uint64_t w = 0;
        for (uint64_t k = 0; k < 5 && b0 + k < nbytes; ++k) w |= (uint64_t)q[b0 + k] << (8 * k);
        outv[got] = (uint32_t)((w >> (bit & 7)) & mask);
      }
      ip += (size_t)nbytes;
    }
  }
  return ip;
}

// ------------------------------------------------------------------ page decoding
struct PageHdr {
  int type = -1, encoding = 0, num_values = 0;
  int32_t uncompressed = 0, compressed = 0;
  int v2_def_len = 0, v2_rep_len = 0;
  bool v2_compressed = true;
};

inline PageHdr parse_page_header(Thrift& t) {
  PageHdr h;
  int id, ty, last = 0;
  while (t.field(id, ty, last)) {
    if (id == 1 && ty == 5) h.type = (int)t.zigzag();
    else if (id == 2 && ty == 5) h.uncompressed = (int32_t)t.zigzag();
    else if (id == 3 && ty == 5) h.compressed = (int32_t)t.zigzag();
    else if ((id == 5 || id == 7 || id == 8) && ty == 12) {
      int fid, fty, flast = 0;
      while (t.field(fid, fty, flast)) {
        if (fid == 1 && fty == 5) h.num_values = (int)t.zigzag();
        else if (id == 5 && fid == 2 && fty == 5) h.encoding = (int)t.zigzag();
        else if (id == 7 && fid == 2 && fty == 5) h.encoding = (int)t.zigzag();
        else if (id == 8 && fid == 4 && fty == 5) h.encoding = (int)t.zigzag();
        else if (id == 8 && fid == 5 && fty == 5) h.v2_def_len = (int)t.zigzag();
        else if (id == 8 && fid == 6 && fty == 5) h.v2_rep_len = (int)t.zigzag();
        else if (id == 8 && fid == 7 && (fty == 1 || fty == 2)) h.v2_compressed = fty == 1;
        else t.skip(fty);
      }
    } else {
      t.skip(ty);
    }
  }
  if (h.compressed < 0 || h.uncompressed < 0 || h.num_values < 0) throw std::runtime_error("parquet: bad page header");
  return h;
}

// Per-thread scratch of the decoder (page decompression, levels, dictionary indices).
struct PqScratch {
  std::vector<uint8_t> page, dict;
  std::vector<uint32_t> levels, idx;
};

inline void fill_null(uint8_t* d, int type, int width) {
  if (type == PT_FLOAT) {
    const float v = std::numeric_limits<float>::quiet_NaN();
    std::memcpy(d, &v, 4);
  } else if (type == PT_DOUBLE) {
    const double v = std::numeric_limits<double>::quiet_NaN();
    std::memcpy(d, &v, 8);
  } else {
    std::memset(d, 0, (size_t)width);
  }
}

// Decode one column chunk of `rows` rows into dst (rows * width bytes; BOOLEAN -> one byte per value).
inline void decode_chunk(const uint8_t* file, size_t fsize, const PqColumn& col, const PqChunk& c, int64_t rows,
                         uint8_t* dst, PqScratch& S) {
  const int width = ptype_width(col.type);
  if (!width || c.type != col.type) throw Unsupported("parquet: column type not decoded natively");
  if (col.repetition == 2) throw Unsupported("parquet: repeated column");
  if (c.codec != 0 && c.codec != 1) throw Unsupported("parquet: codec not decoded natively");
  if (c.num_values != rows) throw std::runtime_error("parquet: chunk value count != row count");
  const int max_def = col.repetition == 1 ? 1 : 0;
  int64_t start = c.data_page_offset;
  if (c.dict_page_offset > 0 && c.dict_page_offset < start) start = c.dict_page_offset;
  if (start < 4 || c.total_compressed < 0 || (uint64_t)start + (uint64_t)c.total_compressed > fsize - 8)
    throw std::runtime_error("parquet: column chunk outside the file");
  size_t pos = (size_t)start;
  const size_t end = (size_t)start + (size_t)c.total_compressed;
  int64_t done = 0;
  int64_t dict_n = -1;
  while (done < rows) {
    if (pos >= end) throw std::runtime_error("parquet: column chunk ends early");
    Thrift t(file + pos, end - pos);
    const PageHdr h = parse_page_header(t);
    pos += t.pos(file + pos);
    if ((size_t)h.compressed > end - pos) throw std::runtime_error("parquet: page outside the chunk");
    const uint8_t* raw = file + pos;
    pos += (size_t)h.compressed;
    if (h.type == 2) {  // dictionary page: PLAIN values
      if (h.encoding != 0 && h.encoding != 2) throw Unsupported("parquet: dictionary encoding");
      const uint8_t* d = raw;
      if (c.codec == 1) {
        snappy_decompress(raw, (size_t)h.compressed, S.dict, (size_t)h.uncompressed);
      } else {
        if (h.compressed != h.uncompressed) throw std::runtime_error("parquet: uncompressed size mismatch");
        S.dict.assign(d, d + h.compressed);
      }
      if (col.type == PT_BOOLEAN) throw Unsupported("parquet: boolean dictionary");
      if ((uint64_t)h.num_values * (uint64_t)width > S.dict.size()) throw std::runtime_error("parquet: short dictionary");
      dict_n = h.num_values;
      continue;
    }
    if (h.type != 0 && h.type != 3) continue;  // index pages etc.
    const int64_t nv = h.num_values;
    if (nv > rows - done) throw std::runtime_error("parquet: more values than rows");
    const uint8_t* body;
    size_t blen;
    const uint8_t* lv = nullptr;
    size_t lvlen = 0;
    if (h.type == 0) {  // data page v1: [def levels (4-byte length + hybrid)] values, all compressed
      if (c.codec == 1) {
        snappy_decompress(raw, (size_t)h.compressed, S.page, (size_t)h.uncompressed);
        body = S.page.data();
        blen = S.page.size();
      } else {
        if (h.compressed != h.uncompressed) throw std::runtime_error("parquet: uncompressed size mismatch");
        body = raw;
        blen = (size_t)h.compressed;
      }
      if (max_def) {
        if (blen < 4) throw std::runtime_error("parquet: levels truncated");
        uint32_t L;
        std::memcpy(&L, body, 4);
        if (L > blen - 4) throw std::runtime_error("parquet: levels truncated");
        lv = body + 4;
        lvlen = L;
        body += 4 + L;
        blen -= 4 + (size_t)L;
      }
    } else {  // data page v2: levels uncompressed in front, values maybe compressed
      if (h.v2_rep_len != 0) throw Unsupported("parquet: repetition levels");
      if (h.v2_def_len < 0 || (size_t)h.v2_def_len > (size_t)h.compressed) throw std::runtime_error("parquet: bad v2 levels");
      if (max_def) {
        lv = raw;
        lvlen = (size_t)h.v2_def_len;
      }
      const uint8_t* vr = raw + h.v2_def_len;
      const size_t vn = (size_t)h.compressed - (size_t)h.v2_def_len;
      if (c.codec == 1 && h.v2_compressed) {
        if (h.uncompressed < h.v2_def_len) throw std::runtime_error("parquet: bad v2 sizes");
        snappy_decompress(vr, vn, S.page, (size_t)h.uncompressed - (size_t)h.v2_def_len);
        body = S.page.data();
        blen = S.page.size();
      } else {
        body = vr;
        blen = vn;
      }
    }
    // definition levels -> count of present values
    int64_t present = nv;
    if (max_def) {
      S.levels.resize((size_t)nv);
      rle_hybrid(lv, lvlen, 1, S.levels.data(), (size_t)nv);
      present = 0;
      for (int64_t i = 0; i < nv; ++i) present += S.levels[(size_t)i] == 1;
    }
    uint8_t* out = dst + (size_t)done * (size_t)width;
    const uint8_t* vals = nullptr;  // PLAIN fixed-width values, or dictionary values via S.idx
    bool dict = false, boolrle = false;
    if (h.encoding == 0) {
      if (col.type == PT_BOOLEAN) {
        if ((uint64_t)(present + 7) / 8 > blen) throw std::runtime_error("parquet: boolean values truncated");
      } else if ((uint64_t)present * (uint64_t)width > blen) {
        throw std::runtime_error("parquet: values truncated");
      }
      vals = body;
    } else if (h.encoding == 2 || h.encoding == 8) {
      if (dict_n < 0) throw std::runtime_error("parquet: dictionary page missing");
      if (blen < 1) throw std::runtime_error("parquet: dictionary indices truncated");
      const int bw = body[0];
      S.idx.resize((size_t)present);
      rle_hybrid(body + 1, blen - 1, bw, S.idx.data(), (size_t)present);
      for (int64_t i = 0; i < present; ++i)
        if (S.idx[(size_t)i] >= (uint64_t)dict_n) throw std::runtime_error("parquet: dictionary index out of range");
      dict = true;
    } else if (h.encoding == 3 && col.type == PT_BOOLEAN) {  // RLE booleans (data page v2)
      if (blen < 4) throw std::runtime_error("parquet: boolean runs truncated");
      uint32_t L;
      std::memcpy(&L, body, 4);
      if (L > blen - 4) throw std::runtime_error("parquet: boolean runs truncated");
      S.idx.resize((size_t)present);
      rle_hybrid(body + 4, L, 1, S.idx.data(), (size_t)present);
      boolrle = true;
    } else {
      throw Unsupported("parquet: value encoding not decoded natively");
    }
    auto value = [&](int64_t k, uint8_t* d) {
      if (boolrle) {
        *d = (uint8_t)S.idx[(size_t)k];
      } else if (dict) {
        std::memcpy(d, S.dict.data() + (size_t)S.idx[(size_t)k] * (size_t)width, (size_t)width);
      } else if (col.type == PT_BOOLEAN) {
        *d = (vals[k >> 3] >> (k & 7)) & 1;
      } else {
        std::memcpy(d, vals + (size_t)k * (size_t)width, (size_t)width);
      }
    };
    if (present == nv && !dict && !boolrle && col.type != PT_BOOLEAN) {
      std::memcpy(out, vals, (size_t)nv * (size_t)width);  // the hot path: one copy into pinned memory
    } else if (present == nv) {
      for (int64_t i = 0; i < nv; ++i) value(i, out + (size_t)i * (size_t)width);
    } else {
      int64_t k = 0;
      for (int64_t i = 0; i < nv; ++i) {
        uint8_t* d = out + (size_t)i * (size_t)width;
        if (S.levels[(size_t)i] == 1) value(k++, d);
        else fill_null(d, col.type, width);
      }
    }
    done += nv;
  }
}

}  // namespace hopsx_io
