#include "consensus_core.h"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <stdexcept>

namespace lwc {

namespace {

bool is_letter(char c) { return c >= 'A' && c <= 'T'; }

template <typename T>
void shuffle(std::vector<T>& v, std::mt19937_64& rng) {
  for (size_t i = v.size(); i > 1; --i) {
    std::uniform_int_distribution<size_t> d(0, i - 1);
    std::swap(v[i - 1], v[d(rng)]);
  }
}

std::vector<char> letters(std::mt19937_64& rng) {
  std::vector<char> v(kNumLetters);
  for (int i = 0; i < kNumLetters; ++i) v[i] = (char)('A' + i);
  shuffle(v, rng);
  return v;
}

// byte offsets of the code points of a UTF-8 string
std::vector<size_t> char_starts(const std::string& s) {
  std::vector<size_t> st;
  st.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i)
    if ((static_cast<unsigned char>(s[i]) & 0xC0) != 0x80) st.push_back(i);
  return st;
}

}  // namespace

const KeyNode* KeyNode::get(char c) const {
  for (const auto& kv : children)
    if (kv.first == c) return kv.second.get();
  return nullptr;
}

KeyTree::KeyTree(int source_len, int max_branch_len, uint64_t seed)
    : source_len_(source_len), max_branch_(max_branch_len) {
  if (source_len < 1) throw std::invalid_argument("KeyTree: need at least one choice");
  if (max_branch_len < 2 || max_branch_len > kNumLetters)
    throw std::invalid_argument("KeyTree: max_branch_len must be in [2, 20]");
  std::mt19937_64 rng(seed);
  std::vector<int> src(source_len);
  std::iota(src.begin(), src.end(), 0);
  shuffle(src, rng);
  root_ = build(rng, src, false);
  collect(root_.get(), "", keys_);
  shuffle(keys_, rng);
}

std::unique_ptr<KeyNode> KeyTree::build(std::mt19937_64& rng, const std::vector<int>& src, bool force) {
  auto node = std::make_unique<KeyNode>();
  const std::vector<char> pfx = letters(rng);
  const int len = (int)src.size();
  const int m = max_branch_;
  if (!force && len <= m) {
    for (int i = 0; i < len; ++i) {
      auto leaf = std::make_unique<KeyNode>();
      leaf->index = src[i];
      node->children.emplace_back(pfx[i], std::move(leaf));
    }
    return node;
  }
  int n = (len + m - 1) / m;
  if (n > m) n = m;
  const int base = len / n, extra = len % n;
  const bool force_sub = base + (extra > 0 ? 1 : 0) > m;
  int count = 0;
  for (int i = 0; i < n; ++i) {
    const int bl = base + (i < extra ? 1 : 0);
    std::vector<int> sub(src.begin() + count, src.begin() + count + bl);
    node->children.emplace_back(pfx[i], build(rng, sub, force_sub));
    count += bl;
  }
  return node;
}

void KeyTree::collect(const KeyNode* n, const std::string& prefix,
                      std::vector<std::pair<std::string, int>>& out) const {
  for (const auto& kv : n->children) {
    std::string k = prefix + "`" + kv.first + "`";
    if (kv.second->is_leaf())
      out.emplace_back(k, kv.second->index);
    else
      collect(kv.second.get(), k, out);
  }
}

int KeyTree::depth() const {
  int d = 0;
  const KeyNode* n = root_.get();
  while (n && !n->is_leaf()) {
    ++d;
    n = n->children.empty() ? nullptr : n->children.front().second.get();
  }
  return d;
}

std::pair<std::string, std::string> KeyTree::regex_patterns() const {
  std::string with, without;
  for (const auto& kv : keys_) {
    if (!with.empty()) {
      with += '|';
      without += '|';
    }
    with += "(" + kv.first + ")";
    without += "(" + kv.first.substr(1, kv.first.size() - 2) + ")";
  }
  return {with, without};
}

std::string KeyTree::find_key(const std::string& content) const {
  // regex alternation of literals, leftmost-first, non-overlapping, keep the last match
  auto scan = [&](bool ticks) -> std::string {
    std::string last;
    size_t i = 0;
    while (i < content.size()) {
      bool hit = false;
      for (const auto& kv : keys_) {
        const std::string pat = ticks ? kv.first : kv.first.substr(1, kv.first.size() - 2);
        if (pat.empty()) continue;
        if (content.compare(i, pat.size(), pat) == 0) {
          last = pat;
          i += pat.size();
          hit = true;
          break;
        }
      }
      if (!hit) ++i;
    }
    return last;
  };
  std::string k = scan(true);
  if (k.empty()) k = scan(false);
  return k;
}

std::optional<std::vector<double>> KeyTree::vote(
    const std::string& content,
    const std::vector<std::pair<std::string, std::vector<std::pair<std::string, double>>>>* logprobs) const {
  const std::string key = find_key(content);
  if (key.empty()) return std::nullopt;
  // final letter and the leaf-parent branch (walk every letter but the last)
  std::vector<char> key_letters;
  for (char c : key)
    if (is_letter(c)) key_letters.push_back(c);
  if (key_letters.empty()) return std::nullopt;
  const char final_c = key_letters.back();
  const KeyNode* branch = root_.get();
  for (size_t i = 0; i + 1 < key_letters.size(); ++i) {
    const KeyNode* nx = branch->get(key_letters[i]);
    if (!nx || nx->is_leaf()) return std::nullopt;
    branch = nx;
  }
  const KeyNode* final_leaf = branch->get(final_c);
  if (!final_leaf || !final_leaf->is_leaf()) return std::nullopt;

  std::vector<double> vote(source_len_, 0.0);
  if (logprobs) {
    const std::string key_rev(key.rbegin(), key.rend());  // key is ASCII
    size_t matched = 0;                                   // chars of key_rev consumed
    int key_lp = -1;
    size_t key_lp_byte = 0;
    bool done = false;
    for (int ti = (int)logprobs->size() - 1; ti >= 0 && !done; --ti) {
      const std::string& tok = (*logprobs)[ti].first;
      const std::vector<size_t> starts = char_starts(tok);
      for (int ci = (int)starts.size() - 1; ci >= 0; --ci) {
        const size_t b0 = starts[ci];
        const size_t clen = (ci + 1 < (int)starts.size() ? starts[ci + 1] : tok.size()) - b0;
        const bool ascii_match = clen == 1 && tok[b0] == key_rev[matched];
        if (ascii_match) {
          ++matched;
          if (key_lp < 0 && tok[b0] == final_c) {
            key_lp = ti;
            key_lp_byte = b0;
          }
          if (matched == key_rev.size()) {
            done = true;
            break;
          }
        } else if (matched != 0) {  // reset (the reference does not re-test this char)
          matched = 0;
          key_lp = -1;
          key_lp_byte = 0;
        }
      }
    }
    if (done && key_lp >= 0) {
      double psum = 0.0;
      for (const auto& alt : (*logprobs)[key_lp].second) {
        const std::string& at = alt.first;
        if (std::isnan(alt.second) || key_lp_byte >= at.size()) continue;
        // must be a char boundary whose char is a single ASCII letter present in the branch
        if ((static_cast<unsigned char>(at[key_lp_byte]) & 0xC0) == 0x80) continue;
        const char c = at[key_lp_byte];
        if (!is_letter(c)) continue;
        const KeyNode* leaf = branch->get(c);
        if (!leaf || !leaf->is_leaf()) continue;
        const double p = std::exp(alt.second);
        vote[leaf->index] += p;
        psum += p;
      }
      if (psum > 0.0) {
        for (double& v : vote) v /= psum;
        return vote;
      }
      std::fill(vote.begin(), vote.end(), 0.0);  // fix: fall back to one-hot
    }
  }
  vote[final_leaf->index] = 1.0;
  return vote;
}

TallyResult tally(const std::vector<std::vector<double>>& votes, const std::vector<double>& weights, int C) {
  if (votes.size() != weights.size()) throw std::invalid_argument("tally: votes/weights length mismatch");
  TallyResult r;
  r.choice_weight.assign(C, 0.0);
  for (size_t l = 0; l < votes.size(); ++l) {
    if (votes[l].empty()) continue;
    if ((int)votes[l].size() != C) throw std::invalid_argument("tally: vote length != choices");
    for (int i = 0; i < C; ++i) r.choice_weight[i] += votes[l][i] * weights[l];
  }
  double sum = 0.0;
  for (double w : r.choice_weight) sum += w;
  r.confidence.assign(C, 0.0);
  for (int i = 0; i < C; ++i) r.confidence[i] = sum > 0.0 ? r.choice_weight[i] / sum : 0.0;
  r.voter_confidence.assign(votes.size(), std::nan(""));
  for (size_t l = 0; l < votes.size(); ++l) {
    if (votes[l].empty()) continue;
    double c = 0.0;
    for (int i = 0; i < C; ++i) c += r.confidence[i] * votes[l][i];
    r.voter_confidence[l] = c;
  }
  return r;
}

std::optional<int> unify_error_codes(const std::vector<int>& codes) {
  if (codes.empty()) return std::nullopt;
  int code = codes[0];
  for (size_t i = 1; i < codes.size(); ++i) {
    const int e = codes[i];
    if (e != code) code = (e >= 400 && e < 500 && code >= 400 && code < 500) ? 400 : 500;
  }
  return code;
}

}  // namespace lwc
