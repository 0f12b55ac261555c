// AddressSanitizer + UndefinedBehaviorSanitizer harness for the hopsx IO parsers (csrc/io/io_core.h).
// SURVEY §5.2 asks for sanitizer builds of the C++ layer; the GPU sanitizer is not available on
// this pool, so the HOST code that parses untrusted files runs here, instrumented:
//   1. round trips: random tf.train.Examples (bytes / float / int64 lists, packed and unpacked)
//      framed as TFRecords, indexed with crc verification and decoded back exactly;
//   2. fuzzing: thousands of mutated inputs (bit flips, byte stores, truncations, splices,
//      random bytes, length fields set to huge values) through index_records, parse_example and
//      the CSV parser.  Every call must either succeed or throw std::runtime_error; any
//      out-of-bounds access, use-after-free, overflow or UB aborts the process (exit != 0).
// Build + run: tests/test_io_asan.py (g++ -fsanitize=address,undefined -fno-sanitize-recover=all).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../csrc/io/io_core.h"

using namespace hopsx_io;

static std::string make_example(std::mt19937_64& rng, std::vector<std::pair<std::string, FeatVal>>& truth) {
  std::string features;
  const int nf = 1 + rng() % 5;
  for (int f = 0; f < nf; ++f) {
    FeatVal fv;
    fv.kind = rng() % 3;
    std::string list, feature;
    const int n = rng() % 6;
    if (fv.kind == 0) {
      for (int i = 0; i < n; ++i) {
        std::string b(rng() % 7, '\0');
        for (auto& c : b) c = (char)(rng() & 0xff);
        fv.b.push_back(b);
        put_len(list, 1, b);
      }
      put_len(feature, 1, list);
    } else if (fv.kind == 1) {
      std::string packed;
      for (int i = 0; i < n; ++i) {
        const float v = (float)((int64_t)(rng() % 2001) - 1000) / 7.f;
        fv.f.push_back(v);
        packed.append((const char*)&v, 4);
      }
      put_len(list, 1, packed);
      put_len(feature, 2, list);
    } else {
      std::string packed;
      for (int i = 0; i < n; ++i) {
        const int64_t v = (int64_t)rng() >> (rng() % 64);
        fv.i.push_back(v);
        put_varint(packed, (uint64_t)v);
      }
      put_len(list, 1, packed);
      put_len(feature, 3, list);
    }
    const std::string name = "f" + std::to_string(f);
    std::string entry;
    put_len(entry, 1, name);
    put_len(entry, 2, feature);
    put_len(features, 1, entry);
    truth.emplace_back(name, fv);
  }
  std::string ex;
  put_len(ex, 1, features);
  return ex;
}

static void mutate(std::mt19937_64& rng, std::string& s) {
  if (s.empty()) {
    s.push_back((char)(rng() & 0xff));
    return;
  }
  switch (rng() % 6) {
    case 0: s[rng() % s.size()] ^= (char)(1u << (rng() % 8)); break;                   // bit flip
    case 1: s[rng() % s.size()] = (char)(rng() & 0xff); break;                          // byte store
    case 2: s.resize(rng() % s.size()); break;                                          // truncation
    case 3: s.insert(rng() % s.size(), std::string(1 + rng() % 4, (char)0xff)); break;  // varint runs
    case 4: {                                                                           // huge length
      const size_t at = rng() % s.size();
      const uint64_t big = ~0ull - (rng() % 64);
      std::string b((const char*)&big, 8);
      s.replace(at, std::min<size_t>(8, s.size() - at), b);
      break;
    }
    default: s.append(s.substr(rng() % s.size(), rng() % 16)); break;                  // splice
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937_64 rng(12345);
  long ok = 0, rejected = 0;
  // 1. round trips
  for (int it = 0; it < 500; ++it) {
    std::vector<std::pair<std::string, FeatVal>> truth;
    const std::string ex = make_example(rng, truth);
    std::string file = frame_record((const uint8_t*)ex.data(), ex.size());
    file += frame_record((const uint8_t*)ex.data(), ex.size());
    auto idx = index_records((const uint8_t*)file.data(), file.size(), true);
    if (idx.size() != 2) return fprintf(stderr, "index_records: %zu records\n", idx.size()), 1;
    auto m = parse_example((const uint8_t*)file.data() + idx[1].first,
                           (const uint8_t*)file.data() + idx[1].first + idx[1].second);
    for (auto& kv : truth) {
      auto f = m.find(kv.first);
      if (f == m.end()) return fprintf(stderr, "missing feature %s\n", kv.first.c_str()), 1;
      if (kv.second.f != f->second.f || kv.second.i != f->second.i || kv.second.b != f->second.b)
        return fprintf(stderr, "round trip mismatch in %s\n", kv.first.c_str()), 1;
    }
  }
  // 2. fuzz
  std::vector<std::pair<std::string, FeatVal>> truth;
  const std::string seed_ex = make_example(rng, truth);
  const std::string seed_file = frame_record((const uint8_t*)seed_ex.data(), seed_ex.size());
  const std::string seed_csv = "a,b,\"c,d\"\n1,2.5,x\n\"3\",,4\r\n5,6,7,8\n";
  for (int it = 0; it < iters; ++it) {
    std::string a = seed_ex, b = seed_file, c = seed_csv;
    const int nm = 1 + rng() % 4;
    for (int k = 0; k < nm; ++k) {
      mutate(rng, a);
      mutate(rng, b);
      mutate(rng, c);
    }
    // exact-size heap copies: a read one byte past the input is an ASan report
    std::vector<uint8_t> ha(a.begin(), a.end()), hb(b.begin(), b.end());
    std::vector<char> hc(c.begin(), c.end());
    try {
      parse_example(ha.data(), ha.data() + ha.size());
      ++ok;
    } catch (const std::runtime_error&) {
      ++rejected;
    }
    for (int verify = 0; verify < 2; ++verify) {
      try {
        auto idx = index_records(hb.data(), hb.size(), verify);
        for (auto& r : idx) parse_example(hb.data() + r.first, hb.data() + r.first + r.second);
        ++ok;
      } catch (const std::runtime_error&) {
        ++rejected;
      }
    }
    CsvTable t = parse_csv_numeric(hc.data(), hc.size(), ',', rng() & 1);
    if (t.vals.size() != t.nrows * t.ncols) return fprintf(stderr, "csv shape mismatch\n"), 1;
  }
  printf("IO_FUZZ_OK iters=%d parsed=%ld rejected=%ld\n", iters, ok, rejected);
  return 0;
}
