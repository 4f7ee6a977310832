// Native Kaldi binary-matrix reader (include/liteasr_io.h).
//
// The reference reads feats.scp entries with its vendored kaldiio (pure Python/numpy,
// liteasr/utils/kaldiio/matio.py:225-554, compression_header.py:17-251) one utterance at a
// time inside DataLoader workers, then pads with torch pad_sequence in the collator
// (liteasr/dataset/asr_dataset.py:115-126).  Here one call decodes a whole minibatch into a
// caller-owned padded float32 buffer (pinned by the caller, so it goes to HBM in one copy),
// on a few host threads, with pread() so threads share nothing.
//
// Decoding arithmetic is float32 in exactly the order numpy evaluates the reference's
// expressions (no contraction: built with -ffp-contract=off), so values are bit-identical.
#include "../../../include/liteasr_io.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

template <typename T>
T bswap(T v) {
  unsigned char b[sizeof(T)];
  std::memcpy(b, &v, sizeof(T));
  std::reverse(b, b + sizeof(T));
  std::memcpy(&v, b, sizeof(T));
  return v;
}

// Sequential reader over one object starting at a byte offset (pread, no shared state).
struct Cursor {
  int fd;
  int64_t pos;
  bool be;
  bool read(void* dst, size_t n) {
    char* p = static_cast<char*>(dst);
    while (n > 0) {
      ssize_t r = pread(fd, p, n, pos);
      if (r <= 0) return false;
      p += r;
      pos += r;
      n -= (size_t)r;
    }
    return true;
  }
  template <typename T>
  bool scalar(T* v) {
    if (!read(v, sizeof(T))) return false;
    if (be) *v = bswap(*v);
    return true;
  }
};

struct Header {
  int kind = 0;
  int64_t rows = 0, cols = 0;  // vectors: cols = 0
  float minv = 0.f, range = 0.f;
  int64_t data_pos = 0;  // first byte after the headers (CM: after the per-column headers)
  int64_t pcol_pos = 0;  // CM: per-column header position
};

int parse_header(Cursor& c, Header* h) {
  char m[2];
  if (!c.read(m, 2)) return fail("ark: truncated object header");
  if (m[0] != '\0' || m[1] != 'B')
    return fail("ark: not a Kaldi binary object (only \"\\0B\" binary matrices/vectors are supported)");
  char tok[8] = {0};
  int n = 0;
  for (;;) {
    char ch;
    if (!c.read(&ch, 1)) return fail("ark: truncated type token");
    if (ch == ' ') break;
    if (n >= 7) return fail("ark: type token too long");
    tok[n++] = ch;
  }
  const std::string t(tok);
  if (t == "CM" || t == "CM2" || t == "CM3") {
    h->kind = t == "CM" ? LASR_ARK_CM : t == "CM2" ? LASR_ARK_CM2 : LASR_ARK_CM3;
    int32_t r, k;
    if (!c.scalar(&h->minv) || !c.scalar(&h->range) || !c.scalar(&r) || !c.scalar(&k))
      return fail("ark: truncated compression header");
    if (r < 0 || k < 0) return fail("ark: negative matrix size");
    h->rows = r;
    h->cols = k;
    if (h->kind == LASR_ARK_CM) {
      h->pcol_pos = c.pos;
      h->data_pos = c.pos + 8 * (int64_t)k;
    } else {
      h->data_pos = c.pos;
    }
    return 0;
  }
  if (t == "FM" || t == "FV" || t == "DM" || t == "DV") {
    h->kind = t == "FM" ? LASR_ARK_FM : t == "FV" ? LASR_ARK_FV : t == "DM" ? LASR_ARK_DM : LASR_ARK_DV;
    char sz;
    int32_t r;
    if (!c.read(&sz, 1) || sz != 4 || !c.scalar(&r)) return fail("ark: bad row-count field");
    h->rows = r;
    h->cols = 0;
    if (t[1] == 'M') {
      int32_t k;
      if (!c.read(&sz, 1) || sz != 4 || !c.scalar(&k)) return fail("ark: bad column-count field");
      h->cols = k;
    }
    if (h->rows < 0 || h->cols < 0) return fail("ark: negative matrix size");
    h->data_pos = c.pos;
    return 0;
  }
  return fail("ark: unsupported type \"" + t + "\" (FM, FV, DM, DV, CM, CM2, CM3)");
}

// GlobalHeader.uint_to_float (compression_header.py:120-122): min + u * range / c, float32.
inline float u2f(float minv, float range, float c, float u) { return minv + (u * range) / c; }

template <typename TO>
int decode(Cursor& c, const Header& h, TO* out, int64_t max_rows, int64_t ld) {
  const int64_t rows = std::min(h.rows, max_rows);
  const int64_t cols = h.cols > 0 ? h.cols : (h.kind == LASR_ARK_FV || h.kind == LASR_ARK_DV ? h.rows : 0);
  const bool vec = h.kind == LASR_ARK_FV || h.kind == LASR_ARK_DV;
  if (vec) {  // one row of length rows
    if (max_rows <= 0) return 0;  // "at most max_rows rows": none
    c.pos = h.data_pos;
    if (h.kind == LASR_ARK_FV) {
      std::vector<float> buf(cols);
      if (!c.read(buf.data(), cols * 4)) return fail("ark: truncated vector data");
      for (int64_t j = 0; j < cols; ++j) out[j] = (TO)(c.be ? bswap(buf[j]) : buf[j]);
    } else {
      std::vector<double> buf(cols);
      if (!c.read(buf.data(), cols * 8)) return fail("ark: truncated vector data");
      for (int64_t j = 0; j < cols; ++j) out[j] = (TO)(c.be ? bswap(buf[j]) : buf[j]);
    }
    return 0;
  }
  switch (h.kind) {
    case LASR_ARK_FM:
    case LASR_ARK_DM: {
      const int64_t es = h.kind == LASR_ARK_FM ? 4 : 8;
      std::vector<char> row(cols * es);
      for (int64_t i = 0; i < rows; ++i) {
        c.pos = h.data_pos + i * cols * es;
        if (!c.read(row.data(), row.size())) return fail("ark: truncated matrix data");
        TO* o = out + i * ld;
        if (es == 4) {
          const float* f = reinterpret_cast<const float*>(row.data());
          for (int64_t j = 0; j < cols; ++j) o[j] = (TO)(c.be ? bswap(f[j]) : f[j]);
        } else {
          const double* f = reinterpret_cast<const double*>(row.data());
          for (int64_t j = 0; j < cols; ++j) o[j] = (TO)(c.be ? bswap(f[j]) : f[j]);
        }
      }
      return 0;
    }
    case LASR_ARK_CM2:
    case LASR_ARK_CM3: {
      const bool two = h.kind == LASR_ARK_CM2;
      const float cst = two ? 65535.0f : 255.0f;
      std::vector<unsigned char> row(cols * (two ? 2 : 1));
      for (int64_t i = 0; i < rows; ++i) {
        c.pos = h.data_pos + i * (int64_t)row.size();
        if (!c.read(row.data(), row.size())) return fail("ark: truncated compressed data");
        TO* o = out + i * ld;
        for (int64_t j = 0; j < cols; ++j) {
          float u;
          if (two) {
            uint16_t v;
            std::memcpy(&v, row.data() + 2 * j, 2);
            u = (float)(c.be ? bswap(v) : v);
          } else {
            u = (float)row[j];
          }
          o[j] = (TO)u2f(h.minv, h.range, cst, u);
        }
      }
      return 0;
    }
    case LASR_ARK_CM: {
      // per-column percentile headers (PerColHeader.read / char_to_float,
      // compression_header.py:140-157, 235-251); data stored column-major [cols][rows]
      std::vector<uint16_t> ph(4 * cols);
      c.pos = h.pcol_pos;
      if (!c.read(ph.data(), ph.size() * 2)) return fail("ark: truncated per-column headers");
      std::vector<unsigned char> col(h.rows);
      const float s1 = (float)(1 / 64.0), s2 = (float)(1 / 128.0), s3 = (float)(1 / 63.0);
      for (int64_t j = 0; j < cols; ++j) {
        float p[4];
        for (int q = 0; q < 4; ++q) {
          uint16_t v = ph[4 * j + q];
          if (c.be) v = bswap(v);
          p[q] = u2f(h.minv, h.range, 65535.0f, (float)v);
        }
        c.pos = h.data_pos + j * h.rows;
        if (!c.read(col.data(), h.rows)) return fail("ark: truncated compressed data");
        const float d1 = p[1] - p[0], d2 = p[2] - p[1], d3 = p[3] - p[2];
        for (int64_t i = 0; i < rows; ++i) {
          const float a = (float)col[i];
          float v;
          if (a <= 64.0f) v = p[0] + (d1 * a) * s1;
          else if (a > 192.0f) v = p[2] + (d3 * (a - 192.0f)) * s3;
          else v = p[1] + (d2 * (a - 64.0f)) * s2;
          out[i * ld + j] = (TO)v;
        }
      }
      return 0;
    }
  }
  return fail("ark: unsupported kind");
}

int open_ro(const char* path) {
  int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  return fd;
}

}  // namespace

extern "C" int lasr_io_version(void) { return 1; }

extern "C" const char* lasr_io_last_error(void) { return g_err.empty() ? nullptr : g_err.c_str(); }

extern "C" int lasr_ark_probe(const char* path, int64_t offset, int big_endian, int64_t* rows,
                              int64_t* cols, int* kind) {
  if (!path || !rows || !cols || !kind) return fail("lasr_ark_probe: null argument");
  int fd = open_ro(path);
  if (fd < 0) return fail(std::string("lasr_ark_probe: cannot open ") + path);
  Cursor c{fd, offset < 0 ? 0 : offset, big_endian != 0};
  Header h;
  int rc = parse_header(c, &h);
  ::close(fd);
  if (rc) return rc;
  *rows = h.rows;
  *cols = h.cols;
  *kind = h.kind;
  return 0;
}

extern "C" int lasr_ark_read(const char* path, int64_t offset, int big_endian, void* out, int out_dtype,
                             int64_t max_rows, int64_t ld, int64_t* rows, int64_t* cols) {
  if (!path || !out) return fail("lasr_ark_read: null argument");
  if (out_dtype != LASR_IO_F32 && out_dtype != LASR_IO_F64) return fail("lasr_ark_read: bad out_dtype");
  int fd = open_ro(path);
  if (fd < 0) return fail(std::string("lasr_ark_read: cannot open ") + path);
  Cursor c{fd, offset < 0 ? 0 : offset, big_endian != 0};
  Header h;
  int rc = parse_header(c, &h);
  if (!rc) {
    const int64_t width = h.cols > 0 ? h.cols : h.rows;
    if (ld < width && !(h.kind == LASR_ARK_FV || h.kind == LASR_ARK_DV)) rc = fail("lasr_ark_read: ld < cols");
    else if (out_dtype == LASR_IO_F32) rc = decode(c, h, static_cast<float*>(out), max_rows, ld);
    else rc = decode(c, h, static_cast<double*>(out), max_rows, ld);
  }
  ::close(fd);
  if (rc) return rc;
  if (rows) *rows = h.rows;
  if (cols) *cols = h.cols;
  return 0;
}

extern "C" int lasr_ark_read_padded(int n, const char* const* paths, const int64_t* offsets, int big_endian,
                                    float* out, int64_t tmax, int64_t feat_dim, int64_t* lens, int nthreads) {
  if (n < 0 || (n > 0 && (!paths || !offsets || !out || !lens))) return fail("lasr_ark_read_padded: bad argument");
  if (n == 0) return 0;
  if (nthreads <= 0) nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  nthreads = std::min(nthreads, n);
  std::atomic<int> next{0};
  std::atomic<int> bad{-1};
  std::vector<std::string> errs(nthreads);
  auto work = [&](int tid) {
    std::unordered_map<std::string, int> fds;  // arks shared by many utterances stay open
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n || bad.load() >= 0) break;
      const std::string p(paths[i]);
      auto it = fds.find(p);
      int fd;
      if (it == fds.end()) {
        fd = open_ro(paths[i]);
        if (fd < 0) {
          errs[tid] = "lasr_ark_read_padded: cannot open " + p;
          bad.store(i);
          break;
        }
        fds.emplace(p, fd);
      } else {
        fd = it->second;
      }
      Cursor c{fd, offsets[i] < 0 ? 0 : offsets[i], big_endian != 0};
      Header h;
      float* dst = out + (int64_t)i * tmax * feat_dim;
      int rc = parse_header(c, &h);
      if (!rc && (h.kind == LASR_ARK_FV || h.kind == LASR_ARK_DV))
        rc = fail("lasr_ark_read_padded: utterance " + std::to_string(i) + " is a vector, not a matrix");
      if (!rc && h.cols != feat_dim)
        rc = fail("lasr_ark_read_padded: utterance " + std::to_string(i) + " has " + std::to_string(h.cols) +
                  " columns, expected " + std::to_string(feat_dim));
      if (!rc && h.rows > tmax)
        rc = fail("lasr_ark_read_padded: utterance " + std::to_string(i) + " has " + std::to_string(h.rows) +
                  " frames > tmax " + std::to_string(tmax));
      if (!rc) rc = decode(c, h, dst, h.rows, feat_dim);
      if (rc) {
        errs[tid] = g_err;
        bad.store(i);
        break;
      }
      std::memset(dst + h.rows * feat_dim, 0, sizeof(float) * (size_t)((tmax - h.rows) * feat_dim));
      lens[i] = h.rows;
    }
    for (auto& kv : fds) ::close(kv.second);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  if (bad.load() >= 0) {
    for (auto& e : errs)
      if (!e.empty()) return fail(e);
    return fail("lasr_ark_read_padded: failed");
  }
  return 0;
}
