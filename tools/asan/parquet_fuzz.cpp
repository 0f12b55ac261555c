// AddressSanitizer + UBSan harness for the native Parquet decoder (csrc/io/parquet_core.h).
// Seeds: Parquet files written by pyarrow in every layout the decoder covers (tests/test_io_asan.py
// passes their paths).  Each seed is decoded as-is (must succeed), then mutated thousands of times
// (bit flips, byte stores, truncations, splices, varint / length fields set to huge values): every
// footer parse and column-chunk decode must either succeed or throw — any out-of-bounds read or
// write, overflow or UB aborts the process.  Output buffers are sized exactly rows * width, so a
// decoder write past its column is an ASan error.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../csrc/io/parquet_core.h"

using namespace hopsx_io;

static int decode_all(const std::string& f, bool must_succeed) {
  const uint8_t* d = (const uint8_t*)f.data();
  int ok = 0;
  try {
    PqMeta m = parse_footer(d, f.size());
    PqScratch S;
    for (const auto& rg : m.row_groups) {
      if (rg.num_rows < 0 || rg.num_rows > (1 << 22)) throw std::runtime_error("rows");
      for (size_t c = 0; c < m.columns.size(); ++c) {
        const int w = ptype_width(m.columns[c].type);
        if (!w) continue;
        std::vector<uint8_t> out((size_t)rg.num_rows * (size_t)w + 1);  // +1: empty chunks
        try {
          decode_chunk(d, f.size(), m.columns[c], rg.chunks[c], rg.num_rows, out.data(), S);
          ++ok;
        } catch (const std::exception&) {
          if (must_succeed) throw;
        }
      }
    }
  } catch (const std::exception& e) {
    if (must_succeed) {
      std::printf("seed failed: %s\n", e.what());
      std::exit(2);
    }
  }
  return ok;
}

int main(int argc, char** argv) {
  if (argc < 3) return 1;
  const long iters = std::atol(argv[1]);
  std::vector<std::string> seeds;
  for (int i = 2; i < argc; ++i) {
    std::ifstream in(argv[i], std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    seeds.push_back(ss.str());
    decode_all(seeds.back(), true);
  }
  std::mt19937_64 rng(12345);
  long decoded = 0;
  for (long it = 0; it < iters; ++it) {
    std::string f = seeds[rng() % seeds.size()];
    const int kind = rng() % 6;
    const int nmut = 1 + rng() % 4;
    for (int k = 0; k < nmut && !f.empty(); ++k) {
      const size_t pos = rng() % f.size();
      switch (kind) {
        case 0: f[pos] ^= (char)(1u << (rng() % 8)); break;
        case 1: f[pos] = (char)(rng() & 0xff); break;
        case 2: f.resize(pos); break;
        case 3: {  // splice a chunk of another seed
          const std::string& o = seeds[rng() % seeds.size()];
          const size_t p2 = rng() % o.size(), n = std::min<size_t>(rng() % 64, o.size() - p2);
          f.replace(pos, std::min(n, f.size() - pos), o, p2, n);
          break;
        }
        case 4: for (int j = 0; j < 4 && pos + j < f.size(); ++j) f[pos + j] = (char)0xff; break;  // huge varint / length
        default: f[pos] = (char)(rng() % 16); break;  // small field headers / types
      }
    }
    decoded += decode_all(f, false);
  }
  std::printf("PARQUET_FUZZ_OK %ld mutated decodes\n", decoded);
  return 0;
}
