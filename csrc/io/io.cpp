// hopsx native data path (_hopsx_io): the C++ replacements for the TF input
// pipeline pieces the reference notebooks rely on (TFRecordDataset + Example
// parsing, mirroredstrategy_mnist_example.ipynb:153-186; CSV readers,
// training_datasets.ipynb:463-526; TensorBoard event files) plus the host side
// of the Parquet/CSV -> HBM path: multi-threaded row gather into pinned memory.
//
//  * crc32c with the SSE4.2 crc32 instruction (TFRecord framing checksums)
//  * TFRecord writer / reader (length, masked crc, payload, masked crc)
//  * tf.train.Example protobuf encode + columnar batch decode
//  * numeric CSV parser -> float32 matrix (empty / non-numeric -> NaN)
//  * gather_rows: shuffled mini-batch assembly by a thread pool
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#if defined(__SSE4_2__)
#include <nmmintrin.h>
#endif

namespace py = pybind11;

// ------------------------------------------------------------------ crc32c
static uint32_t crc_table[256];
static bool crc_init = false;
static void init_crc() {
  if (crc_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    crc_table[i] = c;
  }
  crc_init = true;
}

uint32_t crc32c(const uint8_t* p, size_t n) {
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
  init_crc();
  while (n--) c = crc_table[(c ^ *p++) & 0xFF] ^ (c >> 8);
#endif
  return c ^ 0xFFFFFFFFu;
}

static inline uint32_t masked_crc(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ---------------------------------------------------------------- TFRecord
class TFRecordWriter {
 public:
  explicit TFRecordWriter(const std::string& path, bool append) {
    f_ = fopen(path.c_str(), append ? "ab" : "wb");
    if (!f_) throw std::runtime_error("cannot open " + path);
  }
  ~TFRecordWriter() { close(); }
  void write(py::bytes b) {
    std::string s = b;
    write_raw((const uint8_t*)s.data(), s.size());
  }
  void write_raw(const uint8_t* d, size_t n) {
    if (!f_) throw std::runtime_error("writer closed");
    uint64_t len = n;
    uint8_t hdr[12];
    memcpy(hdr, &len, 8);
    const uint32_t lc = masked_crc(hdr, 8);
    memcpy(hdr + 8, &lc, 4);
    fwrite(hdr, 1, 12, f_);
    fwrite(d, 1, n, f_);
    const uint32_t dc = masked_crc(d, n);
    fwrite(&dc, 1, 4, f_);
  }
  void flush() {
    if (f_) fflush(f_);
  }
  void close() {
    if (f_) {
      fclose(f_);
      f_ = nullptr;
    }
  }

 private:
  FILE* f_ = nullptr;
};

static std::string read_file(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open " + path);
  return std::string((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

static std::vector<std::pair<size_t, size_t>> index_records(const std::string& buf, bool verify) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t pos = 0;
  const uint8_t* b = (const uint8_t*)buf.data();
  while (pos + 12 <= buf.size()) {
    uint64_t len;
    memcpy(&len, b + pos, 8);
    if (verify) {
      uint32_t lc;
      memcpy(&lc, b + pos + 8, 4);
      if (lc != masked_crc(b + pos, 8)) throw std::runtime_error("TFRecord length crc mismatch");
    }
    if (pos + 12 + len + 4 > buf.size()) throw std::runtime_error("truncated TFRecord");
    if (verify) {
      uint32_t dc;
      memcpy(&dc, b + pos + 12 + len, 4);
      if (dc != masked_crc(b + pos + 12, len)) throw std::runtime_error("TFRecord data crc mismatch");
    }
    out.emplace_back(pos + 12, len);
    pos += 12 + len + 4;
  }
  return out;
}

static py::list read_tfrecords(const std::string& path, bool verify) {
  std::string buf = read_file(path);
  auto idx = index_records(buf, verify);
  py::list l;
  for (auto& r : idx) l.append(py::bytes(buf.data() + r.first, r.second));
  return l;
}

// ------------------------------------------------------- protobuf helpers
static inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
static inline void put_key(std::string& o, int field, int wire) { put_varint(o, ((uint64_t)field << 3) | wire); }
static inline void put_len(std::string& o, int field, const std::string& s) {
  put_key(o, field, 2);
  put_varint(o, s.size());
  o += s;
}
static inline uint64_t get_varint(const uint8_t*& p, const uint8_t* end) {
  uint64_t v = 0;
  int sh = 0;
  while (p < end) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) return v;
    sh += 7;
  }
  throw std::runtime_error("truncated varint");
}
static inline void skip_field(const uint8_t*& p, const uint8_t* end, int wire) {
  if (wire == 0) get_varint(p, end);
  else if (wire == 1) p += 8;
  else if (wire == 2) p += get_varint(p, end);
  else if (wire == 5) p += 4;
  else throw std::runtime_error("unsupported wire type");
}

// tf.train.Example: Example{1: Features{1: map<string, Feature>}}; Feature oneof
// {1: BytesList{1: repeated bytes}, 2: FloatList{1: packed float}, 3: Int64List{1: packed int64}}
static py::bytes encode_example(py::dict feats) {
  std::string features;
  for (auto item : feats) {
    const std::string name = py::str(item.first);
    py::tuple kv = py::reinterpret_borrow<py::tuple>(item.second);
    const std::string kind = py::str(kv[0]);
    std::string list, feature;
    if (kind == "float") {
      auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(kv[1]);
      std::string packed((const char*)a.data(), a.size() * 4);
      put_len(list, 1, packed);
      put_len(feature, 2, list);
    } else if (kind == "int64") {
      auto a = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(kv[1]);
      std::string packed;
      for (ssize_t i = 0; i < a.size(); ++i) put_varint(packed, (uint64_t)a.data()[i]);
      put_len(list, 1, packed);
      put_len(feature, 3, list);
    } else if (kind == "bytes") {
      for (auto v : py::reinterpret_borrow<py::list>(kv[1])) {
        std::string s = py::isinstance<py::bytes>(v) ? v.cast<std::string>() : py::str(v).cast<std::string>();
        put_len(list, 1, s);
      }
      put_len(feature, 1, list);
    } else {
      throw std::runtime_error("feature kind must be float/int64/bytes");
    }
    std::string entry;
    put_len(entry, 1, name);
    put_len(entry, 2, feature);
    put_len(features, 1, entry);
  }
  std::string ex;
  put_len(ex, 1, features);
  return py::bytes(ex);
}

struct FeatVal {
  int kind = -1;  // 0 bytes, 1 float, 2 int64
  std::vector<float> f;
  std::vector<int64_t> i;
  std::vector<std::string> b;
};

static void parse_list(const uint8_t* p, const uint8_t* end, int kind, FeatVal& fv) {
  fv.kind = kind;
  while (p < end) {
    const uint64_t key = get_varint(p, end);
    const int field = (int)(key >> 3), wire = (int)(key & 7);
    if (field != 1) {
      skip_field(p, end, wire);
      continue;
    }
    if (kind == 0) {
      const uint64_t n = get_varint(p, end);
      fv.b.emplace_back((const char*)p, n);
      p += n;
    } else if (kind == 1) {
      if (wire == 2) {
        const uint64_t n = get_varint(p, end);
        const size_t cnt = n / 4;
        const size_t off = fv.f.size();
        fv.f.resize(off + cnt);
        memcpy(fv.f.data() + off, p, cnt * 4);
        p += n;
      } else {
        float v;
        memcpy(&v, p, 4);
        p += 4;
        fv.f.push_back(v);
      }
    } else {
      if (wire == 2) {
        const uint64_t n = get_varint(p, end);
        const uint8_t* e = p + n;
        while (p < e) fv.i.push_back((int64_t)get_varint(p, e));
      } else {
        fv.i.push_back((int64_t)get_varint(p, end));
      }
    }
  }
}

static std::unordered_map<std::string, FeatVal> parse_example(const uint8_t* p, const uint8_t* end) {
  std::unordered_map<std::string, FeatVal> out;
  while (p < end) {
    const uint64_t key = get_varint(p, end);
    if ((key >> 3) != 1) {
      skip_field(p, end, key & 7);
      continue;
    }
    const uint64_t flen = get_varint(p, end);
    const uint8_t* fe = p + flen;
    while (p < fe) {  // Features: repeated map entries (field 1)
      const uint64_t k2 = get_varint(p, fe);
      const uint64_t elen = get_varint(p, fe);
      const uint8_t* ee = p + elen;
      if ((k2 >> 3) != 1) {
        p = ee;
        continue;
      }
      std::string name;
      FeatVal fv;
      while (p < ee) {
        const uint64_t k3 = get_varint(p, ee);
        const uint64_t l3 = get_varint(p, ee);
        if ((k3 >> 3) == 1) {
          name.assign((const char*)p, l3);
          p += l3;
        } else if ((k3 >> 3) == 2) {
          const uint8_t* fe2 = p + l3;
          while (p < fe2) {  // Feature oneof
            const uint64_t k4 = get_varint(p, fe2);
            const uint64_t l4 = get_varint(p, fe2);
            const int which = (int)(k4 >> 3);
            parse_list(p, p + l4, which == 1 ? 0 : (which == 2 ? 1 : 2), fv);
            p += l4;
          }
        } else {
          p += l3;
        }
      }
      out.emplace(std::move(name), std::move(fv));
    }
  }
  return out;
}

static py::dict decode_example(py::bytes rec) {
  std::string s = rec;
  auto m = parse_example((const uint8_t*)s.data(), (const uint8_t*)s.data() + s.size());
  py::dict d;
  for (auto& kv : m) {
    if (kv.second.kind == 1) d[py::str(kv.first)] = py::make_tuple("float", py::array_t<float>(kv.second.f.size(), kv.second.f.data()));
    else if (kv.second.kind == 2) d[py::str(kv.first)] = py::make_tuple("int64", py::array_t<int64_t>(kv.second.i.size(), kv.second.i.data()));
    else {
      py::list l;
      for (auto& b : kv.second.b) l.append(py::bytes(b));
      d[py::str(kv.first)] = py::make_tuple("bytes", l);
    }
  }
  return d;
}

// columnar batch decode: schema = [(name, kind 'float'|'int64', length)] -> dict name -> [n, length]
static py::dict decode_examples_columnar(py::list records, py::list schema, int nthreads) {
  const size_t n = records.size();
  std::vector<std::string> recs(n);
  for (size_t i = 0; i < n; ++i) recs[i] = records[i].cast<std::string>();
  struct Col {
    std::string name;
    int kind;
    int len;
    std::vector<float> f;
    std::vector<int64_t> i;
  };
  std::vector<Col> cols;
  for (auto it : schema) {
    py::tuple t = py::reinterpret_borrow<py::tuple>(it);
    Col c;
    c.name = py::str(t[0]);
    c.kind = std::string(py::str(t[1])) == "float" ? 1 : 2;
    c.len = t[2].cast<int>();
    if (c.kind == 1) c.f.assign(n * c.len, NAN);
    else c.i.assign(n * c.len, 0);
    cols.push_back(std::move(c));
  }
  std::atomic<size_t> next{0};
  std::atomic<bool> failed{false};
  std::string err;
  auto work = [&]() {
    try {
      for (size_t r; (r = next.fetch_add(1)) < n && !failed;) {
        auto m = parse_example((const uint8_t*)recs[r].data(), (const uint8_t*)recs[r].data() + recs[r].size());
        for (auto& c : cols) {
          auto it = m.find(c.name);
          if (it == m.end()) continue;
          if (c.kind == 1) {
            const auto& src = it->second.f.empty() && !it->second.i.empty() ? std::vector<float>() : it->second.f;
            if (!it->second.f.empty())
              for (int k = 0; k < c.len && k < (int)src.size(); ++k) c.f[r * c.len + k] = src[k];
            else
              for (int k = 0; k < c.len && k < (int)it->second.i.size(); ++k) c.f[r * c.len + k] = (float)it->second.i[k];
          } else {
            if (!it->second.i.empty())
              for (int k = 0; k < c.len && k < (int)it->second.i.size(); ++k) c.i[r * c.len + k] = it->second.i[k];
            else
              for (int k = 0; k < c.len && k < (int)it->second.f.size(); ++k) c.i[r * c.len + k] = (int64_t)it->second.f[k];
          }
        }
      }
    } catch (std::exception& e) {
      failed = true;
      err = e.what();
    }
  };
  {
    py::gil_scoped_release rel;
    std::vector<std::thread> th;
    const int T = std::max(1, std::min(nthreads, (int)((n + 255) / 256)));
    for (int t = 0; t < T; ++t) th.emplace_back(work);
    for (auto& t : th) t.join();
  }
  if (failed) throw std::runtime_error("Example decode failed: " + err);
  py::dict out;
  for (auto& c : cols) {
    if (c.kind == 1) {
      py::array_t<float> a({(ssize_t)n, (ssize_t)c.len});
      memcpy(a.mutable_data(), c.f.data(), c.f.size() * 4);
      out[py::str(c.name)] = a;
    } else {
      py::array_t<int64_t> a({(ssize_t)n, (ssize_t)c.len});
      memcpy(a.mutable_data(), c.i.data(), c.i.size() * 8);
      out[py::str(c.name)] = a;
    }
  }
  return out;
}

// ---------------------------------------------------------------- CSV
static py::tuple parse_csv_numeric(const std::string& path, char delim, bool header) {
  std::string buf = read_file(path);
  std::vector<std::string> names;
  size_t pos = 0;
  auto next_line = [&](size_t& s, size_t& e) -> bool {
    if (pos >= buf.size()) return false;
    s = pos;
    e = buf.find('\n', pos);
    if (e == std::string::npos) e = buf.size();
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
        names.push_back(cur);
        cur.clear();
      } else cur.push_back(c);
    }
    names.push_back(cur);
  }
  std::vector<float> vals;
  size_t ncols = names.size(), nrows = 0;
  std::string field;
  while (next_line(s, e)) {
    if (e == s) continue;
    size_t col = 0;
    size_t fs = s;
    bool q = false;
    for (size_t i = s; i <= e; ++i) {
      const bool end = (i == e);
      if (!end && buf[i] == '"') q = !q;
      if (end || (buf[i] == delim && !q)) {
        field.assign(buf.data() + fs, i - fs);
        if (field.size() >= 2 && field.front() == '"' && field.back() == '"') field = field.substr(1, field.size() - 2);
        char* ep = nullptr;
        float v = NAN;
        if (!field.empty()) {
          v = strtof(field.c_str(), &ep);
          while (ep && *ep == ' ') ++ep;
          if (!ep || *ep != '\0') v = NAN;
        }
        vals.push_back(v);
        ++col;
        fs = i + 1;
      }
    }
    if (ncols == 0) ncols = col;
    if (col < ncols)
      for (; col < ncols; ++col) vals.push_back(NAN);
    else if (col > ncols)
      vals.resize(vals.size() - (col - ncols));
    ++nrows;
  }
  py::array_t<float> a({(ssize_t)nrows, (ssize_t)ncols});
  if (!vals.empty()) memcpy(a.mutable_data(), vals.data(), vals.size() * 4);
  return py::make_tuple(names, a);
}

// ------------------------------------------------------- batch assembly
// dst[i, :] = src[idx[i], :] for a C-contiguous 2-D byte view, by a thread pool
static void gather_rows(py::array src, py::array_t<int64_t, py::array::c_style | py::array::forcecast> idx,
                        py::array dst, int nthreads) {
  if (src.ndim() < 1 || dst.ndim() < 1) throw std::runtime_error("arrays must be >= 1-D");
  const size_t row_bytes = src.ndim() == 1 ? src.itemsize() : (size_t)src.strides(0);
  const size_t drow = dst.ndim() == 1 ? dst.itemsize() : (size_t)dst.strides(0);
  if (row_bytes != drow) throw std::runtime_error("row size mismatch");
  if (!(src.flags() & py::array::c_style) || !(dst.flags() & py::array::c_style))
    throw std::runtime_error("arrays must be C-contiguous");
  const int64_t* ix = idx.data();
  const size_t n = idx.size();
  if ((size_t)dst.shape(0) < n) throw std::runtime_error("dst too small");
  const size_t nsrc = src.shape(0);
  for (size_t i = 0; i < n; ++i)
    if (ix[i] < 0 || (size_t)ix[i] >= nsrc) throw std::runtime_error("index out of range");
  const char* sp = (const char*)src.data();
  char* dp = (char*)dst.mutable_data();
  py::gil_scoped_release rel;
  const int T = std::max(1, std::min(nthreads, (int)(n / 512 + 1)));
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([=]() {
      for (size_t i = t; i < n; i += T) memcpy(dp + i * row_bytes, sp + (size_t)ix[i] * row_bytes, row_bytes);
    });
  for (auto& x : th) x.join();
}

PYBIND11_MODULE(_hopsx_io, m) {
  m.doc() = "hopsx native data path: TFRecord/Example/CSV codecs and batch assembly";
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c((const uint8_t*)s.data(), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return masked_crc((const uint8_t*)s.data(), s.size());
  });
  py::class_<TFRecordWriter>(m, "TFRecordWriter")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("append") = false)
      .def("write", &TFRecordWriter::write)
      .def("flush", &TFRecordWriter::flush)
      .def("close", &TFRecordWriter::close)
      .def("__enter__", [](TFRecordWriter& w) -> TFRecordWriter& { return w; })
      .def("__exit__", [](TFRecordWriter& w, py::args) { w.close(); });
  m.def("read_tfrecords", &read_tfrecords, py::arg("path"), py::arg("verify") = true);
  m.def("encode_example", &encode_example);
  m.def("decode_example", &decode_example);
  m.def("decode_examples_columnar", &decode_examples_columnar, py::arg("records"), py::arg("schema"),
        py::arg("nthreads") = 8);
  m.def("parse_csv_numeric", &parse_csv_numeric, py::arg("path"), py::arg("delimiter") = ',', py::arg("header") = true);
  m.def("gather_rows", &gather_rows, py::arg("src"), py::arg("idx"), py::arg("dst"), py::arg("nthreads") = 8);
}
