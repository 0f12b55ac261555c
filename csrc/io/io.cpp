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
//  * ParquetFile: native Parquet column decode (parquet_core.h) of mmapped files straight into the
//    pinned staging ring of the Parquet -> HBM reader, GIL released
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "io_core.h"  // the parsers (bounds-checked, no Python types; fuzzed under ASan)
#include "parquet_core.h"

namespace py = pybind11;
using hopsx_io::crc32c;
using hopsx_io::FeatVal;
using hopsx_io::masked_crc;
using hopsx_io::parse_example;
using hopsx_io::put_len;
using hopsx_io::put_varint;

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
    const std::string fr = hopsx_io::frame_record(d, n);
    if (fwrite(fr.data(), 1, fr.size(), f_) != fr.size()) throw std::runtime_error("TFRecord write failed");
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

static py::list read_tfrecords(const std::string& path, bool verify) {
  std::string buf = read_file(path);
  auto idx = hopsx_io::index_records((const uint8_t*)buf.data(), buf.size(), verify);
  py::list l;
  for (auto& r : idx) l.append(py::bytes(buf.data() + r.first, r.second));
  return l;
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

// Columnar TFRecord writer: one tf.train.Example per row from whole columns (the training-dataset
// writer's hot loop).  columns = [(name, kind, data)]: kind 'float' / 'int64' with a 1-D numpy array
// of n values, or 'bytes' with a list of n bytes/str.  Rows are encoded + framed by `nthreads`
// threads into per-thread buffers (contiguous row ranges) and written in row order.
static long write_tfrecord_columnar(const std::string& path, py::list columns, long n, int nthreads) {
  struct Col {
    std::string key;  // pre-encoded "name" field of the feature-map entry
    int kind;         // 0 float, 1 int64, 2 bytes
    const float* f = nullptr;
    const int64_t* i = nullptr;
    std::vector<std::string> b;
  };
  std::vector<Col> cols;
  std::vector<py::object> keep;  // keep the numpy buffers alive
  for (auto c : columns) {
    py::tuple t = py::reinterpret_borrow<py::tuple>(c);
    Col col;
    const std::string name = py::str(t[0]);
    put_len(col.key, 1, name);
    const std::string kind = py::str(t[1]);
    if (kind == "float") {
      auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(t[2]);
      if (!a || a.size() != n) throw std::runtime_error("float column " + name + " must have n values");
      col.kind = 0;
      col.f = a.data();
      keep.push_back(a);
    } else if (kind == "int64") {
      auto a = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(t[2]);
      if (!a || a.size() != n) throw std::runtime_error("int64 column " + name + " must have n values");
      col.kind = 1;
      col.i = a.data();
      keep.push_back(a);
    } else if (kind == "bytes") {
      col.kind = 2;
      py::list l = py::reinterpret_borrow<py::list>(t[2]);
      if ((long)l.size() != n) throw std::runtime_error("bytes column " + name + " must have n values");
      col.b.reserve(n);
      for (auto v : l) col.b.push_back(py::isinstance<py::bytes>(v) ? v.cast<std::string>() : py::str(v).cast<std::string>());
    } else {
      throw std::runtime_error("column kind must be float/int64/bytes");
    }
    cols.push_back(std::move(col));
  }
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + path);
  const int T = std::max(1, std::min(nthreads, (int)std::max(1L, n / 1024)));
  std::vector<std::string> out(T);
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      th.emplace_back([&, t] {
        const long lo = n * t / T, hi = n * (t + 1) / T;
        std::string& o = out[t];
        std::string features, entry, feature, list, packed, ex;
        for (long r = lo; r < hi; ++r) {
          features.clear();
          for (const Col& c : cols) {
            list.clear();
            feature.clear();
            if (c.kind == 0) {
              packed.assign((const char*)(c.f + r), 4);
              put_len(list, 1, packed);
              put_len(feature, 2, list);
            } else if (c.kind == 1) {
              packed.clear();
              put_varint(packed, (uint64_t)c.i[r]);
              put_len(list, 1, packed);
              put_len(feature, 3, list);
            } else {
              put_len(list, 1, c.b[r]);
              put_len(feature, 1, list);
            }
            entry = c.key;
            put_len(entry, 2, feature);
            put_len(features, 1, entry);
          }
          ex.clear();
          put_len(ex, 1, features);
          o += hopsx_io::frame_record((const uint8_t*)ex.data(), ex.size());
        }
      });
    }
    for (auto& x : th) x.join();
  }
  long bytes = 0;
  for (auto& o : out) {
    if (fwrite(o.data(), 1, o.size(), f) != o.size()) {
      fclose(f);
      throw std::runtime_error("TFRecord write failed");
    }
    bytes += (long)o.size();
  }
  fclose(f);
  return bytes;
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
    std::vector<uint8_t> u;  // kind 3: the first bytes value, fixed length (e.g. a raw uint8 image)
  };
  std::vector<Col> cols;
  for (auto it : schema) {
    py::tuple t = py::reinterpret_borrow<py::tuple>(it);
    Col c;
    c.name = py::str(t[0]);
    const std::string k = py::str(t[1]);
    c.kind = k == "float" ? 1 : (k == "bytes" ? 3 : 2);
    c.len = t[2].cast<int>();
    if (c.len < 0) throw std::runtime_error("column length must be >= 0");
    if (c.kind == 1) c.f.assign(n * c.len, NAN);
    else if (c.kind == 3) c.u.assign(n * c.len, 0);
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
          if (c.kind == 3) {
            if (it->second.b.empty()) continue;
            const std::string& v = it->second.b[0];
            if ((int)v.size() != c.len) throw std::runtime_error("bytes feature " + c.name + " has the wrong length");
            memcpy(c.u.data() + r * c.len, v.data(), c.len);
            continue;
          }
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
    } else if (c.kind == 3) {
      py::array_t<uint8_t> a({(ssize_t)n, (ssize_t)c.len});
      if (!c.u.empty()) memcpy(a.mutable_data(), c.u.data(), c.u.size());
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
  const std::string buf = read_file(path);
  hopsx_io::CsvTable t = hopsx_io::parse_csv_numeric(buf.data(), buf.size(), delim, header);
  py::array_t<float> a({(ssize_t)t.nrows, (ssize_t)t.ncols});
  if (!t.vals.empty()) memcpy(a.mutable_data(), t.vals.data(), t.vals.size() * 4);
  return py::make_tuple(t.names, a);
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

// ---------------------------------------------------------------- Parquet
// A read-only mapping of one Parquet file + its parsed footer.  decode() writes the selected columns
// of one row group into caller-owned (pinned) memory; many threads may decode one file at once.
class PqFile {
 public:
  explicit PqFile(const std::string& path) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) {
      ::close(fd_);
      throw std::runtime_error("cannot stat " + path);
    }
    size_ = (size_t)st.st_size;
    if (size_ < 12) {
      ::close(fd_);
      throw std::runtime_error("parquet: file too small: " + path);
    }
    void* p = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) {
      ::close(fd_);
      throw std::runtime_error("cannot mmap " + path);
    }
    data_ = (const uint8_t*)p;
    ::close(fd_);  // the mapping outlives the descriptor: no fd held per cached file
    fd_ = -1;
    madvise(p, size_, MADV_SEQUENTIAL);
    try {
      meta_ = hopsx_io::parse_footer(data_, size_);
    } catch (...) {
      munmap(p, size_);
      throw;
    }
  }
  ~PqFile() {
    if (data_) munmap((void*)data_, size_);
    if (fd_ >= 0) ::close(fd_);
  }
  py::dict meta() const {
    py::dict d;
    d["num_rows"] = meta_.num_rows;
    py::list cols, rgs;
    for (const auto& c : meta_.columns) cols.append(py::make_tuple(c.name, c.type, c.repetition, c.plain));
    for (const auto& rg : meta_.row_groups) {
      py::list ch;
      for (const auto& c : rg.chunks) ch.append(py::make_tuple(c.type, c.codec, c.num_values, c.total_compressed));
      rgs.append(py::make_tuple(rg.num_rows, ch));
    }
    d["columns"] = cols;
    d["row_groups"] = rgs;
    return d;
  }
  // columns: leaf indices; dst: host address; offsets: byte offset of each column's values.
  void decode(int rg, std::vector<int> columns, uintptr_t dst, std::vector<int64_t> offsets) const {
    if (rg < 0 || rg >= (int)meta_.row_groups.size()) throw std::out_of_range("row group");
    if (columns.size() != offsets.size()) throw std::invalid_argument("columns / offsets");
    const auto& g = meta_.row_groups[(size_t)rg];
    for (int c : columns)
      if (c < 0 || c >= (int)meta_.columns.size()) throw std::out_of_range("column");
    py::gil_scoped_release nogil;
    thread_local hopsx_io::PqScratch S;
    for (size_t k = 0; k < columns.size(); ++k) {
      const int c = columns[k];
      hopsx_io::decode_chunk(data_, size_, meta_.columns[(size_t)c], g.chunks[(size_t)c], g.num_rows,
                             (uint8_t*)dst + offsets[k], S);
    }
  }

 private:
  std::string path_;
  int fd_ = -1;
  const uint8_t* data_ = nullptr;
  size_t size_ = 0;
  hopsx_io::PqMeta meta_;
};

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
  m.def("write_tfrecord_columnar", &write_tfrecord_columnar, py::arg("path"), py::arg("columns"), py::arg("n"),
        py::arg("nthreads") = 8);
  m.def("decode_example", &decode_example);
  m.def("decode_examples_columnar", &decode_examples_columnar, py::arg("records"), py::arg("schema"),
        py::arg("nthreads") = 8);
  m.def("parse_csv_numeric", &parse_csv_numeric, py::arg("path"), py::arg("delimiter") = ',', py::arg("header") = true);
  py::register_exception<hopsx_io::Unsupported>(m, "ParquetUnsupported");
  py::class_<PqFile>(m, "ParquetFile")
      .def(py::init<const std::string&>())
      .def("meta", &PqFile::meta)
      .def("decode", &PqFile::decode, py::arg("row_group"), py::arg("columns"), py::arg("dst"), py::arg("offsets"));
  m.def("gather_rows", &gather_rows, py::arg("src"), py::arg("idx"), py::arg("dst"), py::arg("nthreads") = 8);
}
