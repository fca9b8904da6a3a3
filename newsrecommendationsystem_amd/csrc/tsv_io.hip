// Host-side readers of the eval split files (src/evaluate.py:55-71,133-157;
// formats: src/data_preprocess.py:205,239 for news_parsed.tsv, raw MIND
// behaviors.tsv), for the MIND id form. One pass over the file bytes in C++
// replaces the per-line Python split, the 73 k Impression objects and the
// joined-string numeric parses of data.py (EvalPlan: evaluate() at the
// MIND-small-dev shape was host-bound, ~0.5 s of host work for 15 ms of GPU
// passes).
//
// The readers accept exactly the plain form whose values the Python readers
// would produce through their numeric fast paths (data.read_behaviors +
// candidate_rows_numeric / history_rows_numeric, data.read_news_parsed +
// _parse_titles + numeric_news_index); on anything else (a '\r', a non-ASCII
// byte, a cell not in the plain form) they return NRMS_ERR_UNSUPPORTED and
// the caller takes the Python path, which handles every form and raises the
// reference's errors. No device memory, no stream: plain host functions.
#include "nrms_common.hpp"

#include <cstring>
#include <string_view>
#include <unordered_map>

namespace nrms {
namespace {

constexpr int kMaxIdDigits = 18;   // N<digits> ids parse exactly into int64

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// "N<digits>" at p (no leading zero unless the id is "N0"): the number, or -1
inline int64_t parse_nid(const char* p, const char* e, const char** next) {
  if (p >= e || *p != 'N') return -1;
  ++p;
  const char* d0 = p;
  int64_t v = 0;
  while (p < e && is_digit(*p)) {
    v = v * 10 + (*p - '0');
    ++p;
  }
  const int64_t nd = p - d0;
  if (nd == 0 || nd > kMaxIdDigits || (nd > 1 && *d0 == '0')) return -1;
  *next = p;
  return v;
}

struct Line {
  const char* f[5];   // column starts
  const char* g[5];   // column ends
  int n;              // columns found (at most 5 recorded)
};

// Splits [p, e) (one line, no '\n') into its first five tab-separated columns.
inline Line split_line(const char* p, const char* e) {
  Line ln;
  ln.n = 0;
  while (ln.n < 5) {
    const char* q = static_cast<const char*>(memchr(p, '\t', (size_t)(e - p)));
    ln.f[ln.n] = p;
    ln.g[ln.n] = q ? q : e;
    ++ln.n;
    if (!q) break;
    p = q + 1;
  }
  return ln;
}

// One pass over the bytes: whether they are all ASCII without '\r', '\v',
// '\f' (the Python path decides those cases), and the counts of '\n', '-'
// and 'N'. Byte counters in blocks of 255 (branch-free: it vectorises).
bool scan_bytes(const char* buf, int64_t len, int64_t* n_nl, int64_t* n_dash, int64_t* n_N) {
  unsigned bad = 0;
  int64_t a = 0, b = 0, c = 0;
  for (int64_t i0 = 0; i0 < len; i0 += 255) {
    const int64_t i1 = i0 + 255 < len ? i0 + 255 : len;
    uint8_t ca = 0, cb = 0, cc = 0, bb = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const uint8_t x = (uint8_t)buf[i];
      bb |= (uint8_t)((x >= 0x80) | (x == '\r') | (x == '\v') | (x == '\f'));
      ca += (uint8_t)(x == '\n');
      cb += (uint8_t)(x == '-');
      cc += (uint8_t)(x == 'N');
    }
    bad |= bb;
    a += ca;
    b += cb;
    c += cc;
  }
  *n_nl = a;
  *n_dash = b;
  *n_N = c;
  return bad == 0;
}

bool plain_bytes(const char* buf, int64_t len) {
  int64_t a, b, c;
  return scan_bytes(buf, len, &a, &b, &c);
}

template <typename F>
void for_each_line(const char* buf, int64_t len, F&& f) {
  const char* p = buf;
  const char* end = buf + len;
  while (p < end) {
    const char* q = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    if (!q) q = end;
    if (q > p) f(p, q);   // (empty lines are skipped, as data.read_behaviors)
    p = q + 1;
  }
}

// impressions cell "N<id>-<label> N<id>-<label> ...": tokens, or -1
template <typename Emit>
int64_t parse_impressions(const char* p, const char* e, Emit&& emit) {
  if (p == e) return -1;
  int64_t n = 0;
  while (true) {
    const char* q;
    const int64_t id = parse_nid(p, e, &q);
    if (id < 0 || q >= e || *q != '-') return -1;
    p = q + 1;
    const char* d0 = p;
    int64_t lab = 0;
    while (p < e && is_digit(*p)) {
      lab = lab * 10 + (*p - '0');
      ++p;
    }
    if (p == d0 || p - d0 > 9) return -1;
    emit(id, (int32_t)lab);
    ++n;
    if (p == e) return n;
    if (*p != ' ' || p + 1 == e) return -1;   // single spaces, no trailing one
    ++p;
  }
}

// history cell (stripped of spaces, data.history_rows_numeric): "N<id> N<id> ..." or blank
template <typename Emit>
int64_t parse_history(const char* p, const char* e, Emit&& emit) {
  while (p < e && *p == ' ') ++p;
  while (e > p && e[-1] == ' ') --e;
  int64_t n = 0;
  while (p < e) {
    const char* q;
    const int64_t id = parse_nid(p, e, &q);
    if (id < 0) return -1;
    emit(id);
    ++n;
    p = q;
    if (p == e) break;
    if (*p != ' ' || p + 1 == e || p[1] == ' ') return -1;
    ++p;
  }
  return n;
}

}  // namespace
}  // namespace nrms

using namespace nrms;

int32_t nrms_behaviors_scan(const char* buf, int64_t len, int64_t* counts) {
  if (len < 0 || (len > 0 && !buf) || !counts) return NRMS_ERR_INVALID_ARG;
  // upper bounds: a line per '\n' (+ 1), a candidate token per '-', an id per 'N'
  int64_t nl, dash, nn;
  if (!scan_bytes(buf, len, &nl, &dash, &nn)) return NRMS_ERR_UNSUPPORTED;
  counts[0] = nl + 1;
  counts[1] = dash;
  counts[2] = nn;
  return NRMS_OK;
}

int32_t nrms_behaviors_parse(const char* buf, int64_t len, const int64_t* capacity, int64_t* counts,
                             int64_t* fields, int64_t* cand_num, int32_t* labels, int64_t* cand_count,
                             int64_t* hist_num, int64_t* hist_count, int64_t* hist_user) {
  if (len < 0 || (len > 0 && !buf) || !capacity || !counts) return NRMS_ERR_INVALID_ARG;
  const int64_t cap_lines = capacity[0], cap_cand = capacity[1], cap_hist = capacity[2];
  if (cap_lines < 0 || cap_cand < 0 || cap_hist < 0) return NRMS_ERR_INVALID_ARG;
  if ((cap_lines && (!fields || !cand_count || !hist_count || !hist_user)) || (cap_cand && (!cand_num || !labels)) ||
      (cap_hist && !hist_num))
    return NRMS_ERR_INVALID_ARG;
  // the same byte check as nrms_behaviors_scan ('\r', '\v', '\f', non-ASCII:
  // outside the plain MIND form -> the Python readers), so a caller that skips
  // the scan cannot get such columns accepted
  if (!plain_bytes(buf, len)) return NRMS_ERR_UNSUPPORTED;
  // the user key is the history string as data.read_behaviors keeps it (an
  // empty field becomes " "), users numbered in first-seen order (EvalPlan)
  std::unordered_map<std::string_view, int64_t> users;
  users.reserve((size_t)(cap_lines > 0 ? cap_lines : 1));
  static const char kBlank[] = " ";
  int64_t k = 0, nc = 0, nh = 0;
  int32_t st = NRMS_OK;
  for_each_line(buf, len, [&](const char* p, const char* e) {
    if (st != NRMS_OK) return;
    if (k >= cap_lines) { st = NRMS_ERR_WORKSPACE; return; }
    const Line ln = split_line(p, e);
    if (ln.n < 5) { st = NRMS_ERR_UNSUPPORTED; return; }
    for (int c = 0; c < 5; ++c) {
      fields[10 * k + 2 * c] = ln.f[c] - buf;
      fields[10 * k + 2 * c + 1] = ln.g[c] - buf;
    }
    const int64_t c = parse_impressions(ln.f[4], ln.g[4], [&](int64_t id, int32_t lab) {
      if (nc < cap_cand) {
        cand_num[nc] = id;
        labels[nc] = lab;
      }
      ++nc;
    });
    const int64_t h = parse_history(ln.f[3], ln.g[3], [&](int64_t id) {
      if (nh < cap_hist) hist_num[nh] = id;
      ++nh;
    });
    if (c < 0 || h < 0) { st = NRMS_ERR_UNSUPPORTED; return; }
    if (nc > cap_cand || nh > cap_hist) { st = NRMS_ERR_WORKSPACE; return; }
    cand_count[k] = c;
    hist_count[k] = h;
    const std::string_view key = ln.g[3] > ln.f[3] ? std::string_view(ln.f[3], (size_t)(ln.g[3] - ln.f[3]))
                                                   : std::string_view(kBlank, 1);
    hist_user[k] = users.emplace(key, (int64_t)users.size()).first->second;
    ++k;
  });
  counts[0] = k;
  counts[1] = nc;
  counts[2] = nh;
  counts[3] = (int64_t)users.size();
  return st;
}

// news_parsed.tsv: header with "id" and "title" columns; every row's title a
// list literal of exactly L ints "[a, b, ...]" (spaces around the ints
// allowed), and its id N<digits>.
int32_t nrms_news_parse(const char* buf, int64_t len, int32_t L, int64_t* n_rows, int64_t* ids,
                        int64_t* id_spans, int64_t* titles, int64_t capacity) {
  if (len < 0 || (len > 0 && !buf) || L <= 0 || !n_rows || capacity < 0) return NRMS_ERR_INVALID_ARG;
  if (!plain_bytes(buf, len)) return NRMS_ERR_UNSUPPORTED;
  const char* end = buf + len;
  const char* p = buf;
  const char* q = p;
  while (q < end && *q != '\n') ++q;
  // header columns (csv.reader, QUOTE_NONE: fields split on tabs)
  int ci = -1, ct = -1, col = 0;
  {
    const char* s = p;
    for (const char* r = p;; ++r) {
      if (r == q || *r == '\t') {
        const std::string_view f(s, (size_t)(r - s));
        if (f == "id" && ci < 0) ci = col;
        if (f == "title" && ct < 0) ct = col;
        ++col;
        if (r == q) break;
        s = r + 1;
      }
    }
  }
  if (ci < 0 || ct < 0) return NRMS_ERR_UNSUPPORTED;
  int64_t n = 0;
  p = q < end ? q + 1 : end;
  while (p < end) {
    q = p;
    while (q < end && *q != '\n') ++q;
    if (q == p) return NRMS_ERR_UNSUPPORTED;   // (an empty row: the Python reader decides)
    const char* fs[2] = {nullptr, nullptr};
    const char* fe[2] = {nullptr, nullptr};
    const char* s = p;
    col = 0;
    for (const char* r = p;; ++r) {
      if (r == q || *r == '\t') {
        if (col == ci) { fs[0] = s; fe[0] = r; }
        if (col == ct) { fs[1] = s; fe[1] = r; }
        ++col;
        if (r == q) break;
        s = r + 1;
      }
    }
    if (!fs[0] || !fs[1]) return NRMS_ERR_UNSUPPORTED;
    const char* nx;
    const int64_t id = parse_nid(fs[0], fe[0], &nx);
    if (id < 0 || nx != fe[0]) return NRMS_ERR_UNSUPPORTED;
    // the title literal
    const char* t = fs[1];
    const char* te = fe[1];
    while (t < te && *t == ' ') ++t;
    while (te > t && te[-1] == ' ') --te;
    if (te - t < 2 || *t != '[' || te[-1] != ']') return NRMS_ERR_UNSUPPORTED;
    ++t;
    --te;
    if (n < capacity) {
      ids[n] = id;
      id_spans[2 * n] = fs[0] - buf;
      id_spans[2 * n + 1] = fe[0] - buf;
    }
    for (int i = 0; i < L; ++i) {
      while (t < te && *t == ' ') ++t;
      bool neg = false;
      if (t < te && (*t == '-' || *t == '+')) { neg = *t == '-'; ++t; }
      const char* d0 = t;
      int64_t v = 0;
      while (t < te && is_digit(*t)) {
        v = v * 10 + (*t - '0');
        ++t;
      }
      if (t == d0 || t - d0 > kMaxIdDigits) return NRMS_ERR_UNSUPPORTED;
      while (t < te && *t == ' ') ++t;
      if (i + 1 < L) {
        if (t >= te || *t != ',') return NRMS_ERR_UNSUPPORTED;
        ++t;
      } else if (t != te) {
        return NRMS_ERR_UNSUPPORTED;
      }
      if (n < capacity) titles[n * L + i] = neg ? -v : v;
    }
    ++n;
    p = q + 1;
  }
  *n_rows = n;
  return n > capacity ? NRMS_ERR_WORKSPACE : NRMS_OK;
}
