// Native similarity gate of the evolution loop.
//
// The reference drops a child program when some population member that
// scores at least as well is textually similar to it:
//   difflib.SequenceMatcher(None, new.strip(), old.strip()).ratio() >= 0.85
// (reference funsearch/funsearch_integration.py, SimpleFunSearch._is_too_similar).
// In pure Python that check costs ~5 ms per pair on 4 kB programs and was the
// largest host cost of a 4-island generation after the device replay.  This is
// an exact re-implementation of CPython's SequenceMatcher for isjunk=None,
// autojunk=True, on code-point sequences: same popular-element pruning, same
// longest-match tie breaking, same recursion, same 2*M/T ratio in double.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace fks {

class SeqMatcher {
 public:
  SeqMatcher(const std::u32string& a, const std::u32string& b) : a_(a), b_(b) {
    const int lb = static_cast<int>(b_.size());
    for (int j = 0; j < lb; ++j) b2j_[b_[j]].push_back(j);
    if (lb >= 200) {  // autojunk: drop elements present in more than 1% + 1 of b
      const size_t ntest = static_cast<size_t>(lb / 100 + 1);
      for (auto it = b2j_.begin(); it != b2j_.end();) {
        if (it->second.size() > ntest) it = b2j_.erase(it); else ++it;
      }
    }
    for (auto& kv : b2j_) {
      if (kv.first < 128) ascii_[kv.first] = &kv.second;
    }
    val_[0].assign(lb, 0); val_[1].assign(lb, 0);
    stamp_[0].assign(lb, -1); stamp_[1].assign(lb, -1);
  }

  /// Upper bound of ratio(): 2 * |multiset(a) & multiset(b)| / (la + lb).
  double quick_ratio() const {
    std::unordered_map<char32_t, int64_t> avail;
    for (char32_t c : b_) ++avail[c];
    int64_t m = 0;
    for (char32_t c : a_) {
      auto it = avail.find(c);
      if (it != avail.end() && it->second > 0) { --it->second; ++m; }
    }
    return ratio_of(m);
  }

  double real_quick_ratio() const {
    return ratio_of(static_cast<int64_t>(a_.size() < b_.size() ? a_.size() : b_.size()));
  }

  double ratio() {
    const int la = static_cast<int>(a_.size()), lb = static_cast<int>(b_.size());
    int64_t matched = 0;
    struct Range { int v[4]; };
    std::vector<Range> stack;
    stack.push_back({{0, la, 0, lb}});
    while (!stack.empty()) {
      auto q = stack.back();
      stack.pop_back();
      int i, j, k;
      longest_match(q.v[0], q.v[1], q.v[2], q.v[3], i, j, k);
      if (k) {
        matched += k;
        if (q.v[0] < i && q.v[2] < j) stack.push_back({{q.v[0], i, q.v[2], j}});
        if (i + k < q.v[1] && j + k < q.v[3]) stack.push_back({{i + k, q.v[1], j + k, q.v[3]}});
      }
    }
    return ratio_of(matched);
  }

  /// ratio() >= t, pruned by the two upper bounds (the same decision).
  bool at_least(double t) {
    if (real_quick_ratio() < t) return false;
    if (quick_ratio() < t) return false;
    return ratio() >= t;
  }

 private:
  double ratio_of(int64_t m) const {
    const int64_t len = static_cast<int64_t>(a_.size() + b_.size());
    return len ? 2.0 * static_cast<double>(m) / static_cast<double>(len) : 1.0;
  }

  const std::vector<int>* positions(char32_t c) const {
    if (c < 128) return ascii_[c];
    auto it = b2j_.find(c);
    return it == b2j_.end() ? nullptr : &it->second;
  }

  // find_longest_match(alo, ahi, blo, bhi) with no junk predicate.  The
  // per-row dict j2len is two stamped arrays: an entry counts only when its
  // stamp is the previous row's id, so nothing is cleared between rows.
  void longest_match(int alo, int ahi, int blo, int bhi, int& bi, int& bj, int& bs) {
    int besti = alo, bestj = blo, bestsize = 0;
    row_ += 2;  // the row before this call's first row was never stamped
    for (int i = alo; i < ahi; ++i, ++row_) {
      const int64_t r = row_;
      const int cur = static_cast<int>(r & 1), prev = cur ^ 1;
      const std::vector<int>* js = positions(a_[i]);
      if (!js) continue;
      for (int j : *js) {
        if (j < blo) continue;
        if (j >= bhi) break;
        int k = 1;
        if (j > 0 && stamp_[prev][j - 1] == r - 1) k += val_[prev][j - 1];
        val_[cur][j] = k;
        stamp_[cur][j] = r;
        if (k > bestsize) { besti = i - k + 1; bestj = j - k + 1; bestsize = k; }
      }
    }
    while (besti > alo && bestj > blo && a_[besti - 1] == b_[bestj - 1]) { --besti; --bestj; ++bestsize; }
    while (besti + bestsize < ahi && bestj + bestsize < bhi && a_[besti + bestsize] == b_[bestj + bestsize]) ++bestsize;
    bi = besti; bj = bestj; bs = bestsize;
  }

  const std::u32string& a_;
  const std::u32string& b_;
  std::unordered_map<char32_t, std::vector<int>> b2j_;
  const std::vector<int>* ascii_[128] = {};
  std::vector<int> val_[2];
  std::vector<int64_t> stamp_[2];
  int64_t row_ = 0;
};

}  // namespace fks
