// Host-side AddressSanitizer / UBSan driver for the two host-only native libraries:
// the Kaldi ark reader (csrc/io/ark_io.cpp) and the CTC prefix beam search
// (csrc/decode/prefix_beam.cpp). Built from their sources with -fsanitize=address,undefined
// (tools/asan/Makefile); tests/test_asan_cpu.py builds and runs it. It writes ark objects of
// every supported kind, reads them back (full, row-limited, padded ld, the threaded padded
// reader), then feeds the reader every truncation and many byte-mutations of those objects
// (each must fail cleanly or succeed inside the caller's probe-sized buffer), and runs the
// beam search over ragged shapes, tiny beams and too-small token caps. Exit 0 = clean.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/liteasr_decode.h"
#include "../../include/liteasr_io.h"

static int g_fail = 0;
#define CHECK(c, ...)                              \
  do {                                             \
    if (!(c)) {                                    \
      std::fprintf(stderr, "CHECK failed: " #c " "); \
      std::fprintf(stderr, __VA_ARGS__);           \
      std::fprintf(stderr, "\n");                  \
      ++g_fail;                                    \
    }                                              \
  } while (0)

static void put(std::string& s, const void* p, size_t n) { s.append(static_cast<const char*>(p), n); }
static void put_i32(std::string& s, int32_t v) {
  const char four = 4;
  put(s, &four, 1);
  put(s, &v, 4);
}

// one binary object ("\0B" + token + sizes + payload) of the given kind
static std::string object(const std::string& tok, int32_t rows, int32_t cols, std::mt19937& rng) {
  std::string s("\0B", 2);
  s += tok + " ";
  std::uniform_real_distribution<float> U(-3.f, 3.f);
  if (tok == "FM" || tok == "DM" || tok == "FV" || tok == "DV") {
    put_i32(s, rows);
    if (tok[1] == 'M') put_i32(s, cols);
    const int64_t n = (int64_t)rows * (tok[1] == 'M' ? cols : 1);
    for (int64_t i = 0; i < n; ++i) {
      if (tok[0] == 'F') {
        const float v = U(rng);
        put(s, &v, 4);
      } else {
        const double v = U(rng);
        put(s, &v, 8);
      }
    }
    return s;
  }
  const float minv = -2.f, range = 4.f;
  put(s, &minv, 4);
  put(s, &range, 4);
  put(s, &rows, 4);
  put(s, &cols, 4);
  if (tok == "CM") {  // per-column percentile headers, then column-major bytes
    for (int c = 0; c < cols; ++c) {
      const uint16_t h[4] = {0, 16000, 48000, 65535};
      put(s, h, 8);
    }
    for (int64_t i = 0; i < (int64_t)rows * cols; ++i) {
      const uint8_t b = (uint8_t)(rng() & 255);
      put(s, &b, 1);
    }
  } else if (tok == "CM2") {
    for (int64_t i = 0; i < (int64_t)rows * cols; ++i) {
      const uint16_t b = (uint16_t)(rng() & 65535);
      put(s, &b, 2);
    }
  } else {
    for (int64_t i = 0; i < (int64_t)rows * cols; ++i) {
      const uint8_t b = (uint8_t)(rng() & 255);
      put(s, &b, 1);
    }
  }
  return s;
}

static void write_file(const std::string& path, const std::string& data) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
}

// probe, then read into exactly the probe-sized buffer (the documented caller contract)
static int probe_read(const std::string& path, int64_t off, int dtype, int64_t max_rows, int64_t ld_extra) {
  int64_t rows = -1, cols = -1;
  int kind = 0;
  if (lasr_ark_probe(path.c_str(), off, 0, &rows, &cols, &kind) != 0) return -1;
  const bool vec = kind == LASR_ARK_FV || kind == LASR_ARK_DV;
  if (rows > (1 << 22) || cols > (1 << 22) || rows * (cols > 0 ? cols : 1) > (1 << 22))
    return -2;  // a mutated size field: not worth allocating
  // a matrix writes min(rows, max_rows) rows of stride ld; a vector is one row of `rows`
  // elements (none when max_rows <= 0)
  const int64_t ld = (vec ? rows : cols) + ld_extra;
  const int64_t r = vec ? (max_rows > 0 ? 1 : 0) : (rows < max_rows ? rows : max_rows);
  const size_t esz = dtype == LASR_IO_F32 ? 4 : 8;
  const size_t need = r > 0 ? (size_t)((r - 1) * ld + (vec ? rows : cols)) : 0;
  std::vector<char> buf((need > 0 ? need : 1) * esz);
  int64_t rr = -1, cc = -1;
  const int rc = lasr_ark_read(path.c_str(), off, 0, buf.data(), dtype, max_rows, ld > 0 ? ld : 1, &rr, &cc);
  if (rc == 0) CHECK(rr == rows && cc == cols, "rows %ld/%ld cols %ld/%ld", (long)rr, (long)rows, (long)cc, (long)cols);
  return rc;
}

static void ark_checks(const std::string& dir) {
  std::mt19937 rng(7);
  const char* toks[] = {"FM", "FV", "DM", "DV", "CM", "CM2", "CM3"};
  std::vector<std::string> objs;
  for (const char* t : toks)
    for (int32_t rows : {0, 1, 7, 33})
      objs.push_back(object(t, rows, std::string(t).substr(0, 1) == "C" || std::string(t)[1] == 'M' ? 5 : 0, rng));
  // one ark holding every object back to back (offsets as in feats.scp)
  std::string ark;
  std::vector<int64_t> offs;
  for (auto& o : objs) {
    ark += "utt" + std::to_string(offs.size()) + " ";
    offs.push_back((int64_t)ark.size());
    ark += o;
  }
  const std::string path = dir + "/all.ark";
  write_file(path, ark);
  for (size_t i = 0; i < objs.size(); ++i)
    for (int dt : {LASR_IO_F32, LASR_IO_F64})
      for (int64_t mr : {(int64_t)1 << 30, (int64_t)3, (int64_t)0}) {
        const int rc = probe_read(path, offs[i], dt, mr, i % 2);
        CHECK(rc == 0, "object %zu dtype %d max_rows %ld: %s", i, dt, (long)mr, lasr_io_last_error());
      }
  // threaded padded reader over the 5-column matrices (every kind except vectors)
  std::vector<const char*> paths;
  std::vector<int64_t> poffs;
  for (size_t i = 0; i < objs.size(); ++i) {
    const std::string t(toks[i / 4]);
    if (t == "FV" || t == "DV") continue;
    paths.push_back(path.c_str());
    poffs.push_back(offs[i]);
  }
  const int n = (int)paths.size();
  std::vector<float> out((size_t)n * 40 * 5);
  std::vector<int64_t> lens(n);
  CHECK(lasr_ark_read_padded(n, paths.data(), poffs.data(), 0, out.data(), 40, 5, lens.data(), 3) == 0, "%s",
        lasr_io_last_error());
  CHECK(lasr_ark_read_padded(n, paths.data(), poffs.data(), 0, out.data(), 8, 5, lens.data(), 3) != 0,
        "tmax below the longest utterance must fail");
  CHECK(lasr_ark_read_padded(n, paths.data(), poffs.data(), 0, out.data(), 40, 4, lens.data(), 2) != 0,
        "wrong feature dimension must fail");
  // every truncation and random byte mutations of every object: fail cleanly or read in bounds
  int fuzz = 0;
  for (size_t i = 0; i < objs.size(); ++i) {
    const std::string& o = objs[i];
    const std::string tp = dir + "/t.ark";
    for (size_t cut = 0; cut < o.size(); cut += (o.size() > 200 ? 7 : 1)) {
      write_file(tp, o.substr(0, cut));
      probe_read(tp, 0, LASR_IO_F32, 1 << 30, 0);
      ++fuzz;
    }
    for (int m = 0; m < 200; ++m) {
      std::string x = o;
      const int nb = 1 + (int)(rng() % 4);
      for (int b = 0; b < nb; ++b) x[rng() % x.size()] = (char)(rng() & 255);
      write_file(tp, x);
      probe_read(tp, 0, m % 2 ? LASR_IO_F32 : LASR_IO_F64, 1 << 30, m % 3);
      ++fuzz;
    }
  }
  CHECK(lasr_ark_probe((dir + "/missing.ark").c_str(), 0, 0, nullptr, nullptr, nullptr) != 0, "missing file");
  std::printf("ark: %zu objects x 2 dtypes x 3 row limits, padded reader, %d truncated/mutated reads\n",
              objs.size(), fuzz);
}

static void decode_checks() {
  std::mt19937 rng(11);
  std::normal_distribution<float> N(0.f, 2.f);
  int runs = 0;
  for (int T : {0, 1, 2, 17, 120})
    for (int k : {1, 3, 10})
      for (int beam : {1, 2, 5, 10})
        for (int64_t cap : {(int64_t)0, (int64_t)3, (int64_t)4096}) {
          const int V = 30;
          std::vector<float> val((size_t)T * k);
          std::vector<int32_t> idx((size_t)T * k);
          for (int t = 0; t < T; ++t) {
            std::vector<int32_t> perm(V);
            for (int v = 0; v < V; ++v) perm[v] = v;
            std::shuffle(perm.begin(), perm.end(), rng);
            std::vector<float> lv(k);
            for (int j = 0; j < k; ++j) lv[j] = N(rng);
            std::sort(lv.begin(), lv.end(), [](float a, float b) { return a > b; });
            float mx = lv[0], s = 0.f;
            for (float v : lv) s += std::exp(v - mx);
            for (int j = 0; j < k; ++j) {
              val[(size_t)t * k + j] = lv[j] - mx - std::log(s);
              idx[(size_t)t * k + j] = perm[j];
            }
          }
          std::vector<int32_t> tok(cap > 0 ? (size_t)cap : 1), len(beam);
          std::vector<double> score(beam);
          const int rc = lasr_ctc_prefix_beam_search(T ? val.data() : nullptr, T ? idx.data() : nullptr, T, k, 0,
                                                     beam, cap > 0 ? tok.data() : nullptr, cap, len.data(),
                                                     score.data());
          CHECK(rc >= 0 || rc == -2, "T %d k %d beam %d cap %ld rc %d: %s", T, k, beam, (long)cap, rc,
                lasr_decode_last_error());
          if (rc >= 0) {
            CHECK(rc >= 1 && rc <= beam, "hypothesis count %d", rc);
            int64_t used = 0;
            for (int h = 0; h < rc; ++h) used += len[h];
            CHECK(used <= cap, "tokens %ld > cap %ld", (long)used, (long)cap);
          }
          ++runs;
        }
  int32_t l = 0;
  double sc = 0;
  CHECK(lasr_ctc_prefix_beam_search(nullptr, nullptr, 5, 1, 0, 1, nullptr, 0, &l, &sc) == -1, "null inputs");
  CHECK(lasr_ctc_prefix_beam_search(nullptr, nullptr, 0, 0, 0, 1, nullptr, 0, &l, &sc) == -1, "k = 0");
  std::printf("decode: %d searches (ragged T, k, beam, token caps)\n", runs);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  ark_checks(dir);
  decode_checks();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host sanitizer checks: clean\n");
  return 0;
}
