// CTC prefix beam search on the host, over per-frame top-k candidates produced on the
// device by lasr_logsoftmax_topk.  Follows liteasr/models/u2.py:218-263 step for step
// (and log_add, u2.py:367-375), in double precision like the reference's Python floats:
//  * next-hypothesis entries are created in the order the reference's defaultdict first
//    touches them (blank: prefix; repeat: prefix then prefix+s; other: prefix+s), which
//    fixes the order ties keep through the stable sort;
//  * log_add: -inf if every argument is -inf, else a_max + log(0 + sum_i exp(a_i - a_max))
//    summed left to right;
//  * each frame keeps the `beam` best by log_add(pb, pnb), stable descending sort.
// Prefixes live in a trie (node = parent + last token), so "prefix + s" is one hash
// lookup and prefix equality is node equality; no per-candidate vector copies.
// Built with -ffp-contract=off so exp/log/add are the plain libm/IEEE operations the
// reference's math.exp / math.log / float + perform.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <unordered_map>
#include <vector>

#include "../../../include/liteasr_decode.h"

namespace {

thread_local char g_err[256] = "";

double log_add(const double* a, int n) {
  bool all_ninf = true;
  for (int i = 0; i < n; ++i) all_ninf = all_ninf && (a[i] == -INFINITY);
  if (all_ninf) return -INFINITY;
  double m = a[0];
  for (int i = 1; i < n; ++i)
    if (a[i] > m) m = a[i];
  // exp(-inf) == 0 and exp(0) == 1 exactly, log(1) == 0: skipping those libm calls
  // leaves every result bit-identical
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += (a[i] == -INFINITY) ? 0.0 : (a[i] == m ? 1.0 : std::exp(a[i] - m));
  return m + (s == 1.0 ? 0.0 : std::log(s));
}

struct Trie {
  std::vector<int32_t> parent{-1}, token{-1}, depth{0};  // node 0 = empty prefix
  std::unordered_map<uint64_t, int32_t> child;
  int32_t extend(int32_t node, int32_t s) {
    const uint64_t key = ((uint64_t)(uint32_t)node << 32) | (uint32_t)s;
    auto it = child.find(key);
    if (it != child.end()) return it->second;
    const int32_t id = (int32_t)parent.size();
    parent.push_back(node);
    token.push_back(s);
    depth.push_back(depth[node] + 1);
    child.emplace(key, id);
    return id;
  }
};

struct Hyp {
  int32_t node;
  double pb, pnb;
};

// Per-frame hypothesis set: node -> slot via frame-stamped arrays (no hashing, no clear)
struct NextHyps {
  std::vector<Hyp> items;  // insertion order
  std::vector<int32_t> stamp, slot;
  int32_t frame = -1;
  void reset(int32_t t) {
    frame = t;
    items.clear();
  }
  Hyp& at(int32_t node) {
    if ((size_t)node >= stamp.size()) {
      stamp.resize((size_t)node * 2 + 64, -1);
      slot.resize(stamp.size());
    }
    if (stamp[node] == frame) return items[slot[node]];
    stamp[node] = frame;
    slot[node] = (int32_t)items.size();
    items.push_back(Hyp{node, -INFINITY, -INFINITY});
    return items.back();
  }
};

}  // namespace

extern "C" const char* lasr_decode_last_error(void) { return g_err; }

extern "C" int lasr_ctc_prefix_beam_search(const float* topk_val, const int32_t* topk_idx, int T,
                                           int k, int blank, int beam, int32_t* out_tok,
                                           int64_t cap_tok, int32_t* out_len,
                                           double* out_score) {
  if (T < 0 || k <= 0 || beam <= 0 || (T > 0 && (topk_val == nullptr || topk_idx == nullptr)) ||
      out_len == nullptr || out_score == nullptr || (cap_tok > 0 && out_tok == nullptr)) {
    std::snprintf(g_err, sizeof g_err, "ctc_prefix_beam_search: bad arguments (T=%d k=%d beam=%d)",
                  T, k, beam);
    return -1;
  }
  Trie trie;
  trie.child.reserve((size_t)T * k * 2 + 16);
  std::vector<Hyp> cur{Hyp{0, 0.0, -INFINITY}};
  NextHyps nxt;
  std::vector<std::pair<double, size_t>> order;
  std::vector<Hyp> kept;
  for (int t = 0; t < T; ++t) {
    nxt.reset(t);
    for (int j = 0; j < k; ++j) {
      const int32_t s = topk_idx[(int64_t)t * k + j];
      const double ps = (double)topk_val[(int64_t)t * k + j];
      for (const Hyp& h : cur) {
        const bool has_last = h.node != 0;
        const int32_t last = has_last ? trie.token[h.node] : 0;
        if (s == blank) {
          Hyp& n = nxt.at(h.node);
          const double a[3] = {n.pb, h.pb + ps, h.pnb + ps};
          n.pb = log_add(a, 3);
        } else if (has_last && s == last) {
          {
            Hyp& n = nxt.at(h.node);
            const double a[2] = {n.pnb, h.pnb + ps};
            n.pnb = log_add(a, 2);
          }
          Hyp& n = nxt.at(trie.extend(h.node, s));
          const double a[2] = {n.pnb, h.pb + ps};
          n.pnb = log_add(a, 2);
        } else {
          Hyp& n = nxt.at(trie.extend(h.node, s));
          const double a[3] = {n.pnb, h.pb + ps, h.pnb + ps};
          n.pnb = log_add(a, 3);
        }
      }
    }
    order.clear();
    for (size_t i = 0; i < nxt.items.size(); ++i) {
      const double a[2] = {nxt.items[i].pb, nxt.items[i].pnb};
      order.emplace_back(log_add(a, 2), i);
    }
    std::stable_sort(order.begin(), order.end(),
                     [](const auto& x, const auto& y) { return x.first > y.first; });
    kept.clear();
    for (size_t i = 0; i < order.size() && (int)i < beam; ++i)
      kept.push_back(nxt.items[order[i].second]);
    cur.swap(kept);
  }
  int64_t used = 0;
  for (const Hyp& h : cur) used += trie.depth[h.node];
  if (used > cap_tok) {
    std::snprintf(g_err, sizeof g_err,
                  "ctc_prefix_beam_search: %lld output tokens exceed capacity %lld",
                  (long long)used, (long long)cap_tok);
    return -2;
  }
  int64_t o = 0;
  for (size_t i = 0; i < cur.size(); ++i) {
    const Hyp& h = cur[i];
    const int32_t n = trie.depth[h.node];
    for (int32_t j = n - 1, v = h.node; j >= 0; --j, v = trie.parent[v]) out_tok[o + j] = trie.token[v];
    o += n;
    out_len[i] = n;
    const double a[2] = {h.pb, h.pnb};
    out_score[i] = log_add(a, 2);
  }
  return (int)cur.size();
}
