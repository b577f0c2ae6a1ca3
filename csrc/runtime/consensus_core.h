// Consensus core (host C++): the voter key prefix tree, vote extraction and the weighted tally.
//
// Behavioural contract (reference, read-only):
//   * SelectPfx / SelectPfxTree     src/score/completions/client.rs:1342-1631
//   * get_vote                      src/score/completions/client.rs:1661-1800
//   * tally + confidence            src/score/completions/client.rs:384-455
// Deliberate fixes of reference quirks:
//   * descent walks the key's letters until it reaches the leaf-parent branch instead of trusting
//     `depth()` of the first child (unequal subtree depths for N > m^3 panicked in the reference);
//   * a logprob match whose top-logprobs hold no sibling letter falls back to the one-hot vote
//     instead of `unreachable!()`.
#pragma once
#include <cstdint>
#include <memory>
#include <optional>
#include <random>
#include <string>
#include <utility>
#include <vector>

namespace lwc {

constexpr int kNumLetters = 20;  // 'A'..'T'

struct KeyNode {
  // leaf: index >= 0, children empty; branch: index = -1, children in insertion order
  int index = -1;
  std::vector<std::pair<char, std::unique_ptr<KeyNode>>> children;
  const KeyNode* get(char c) const;
  bool is_leaf() const { return index >= 0; }
};

class KeyTree {
 public:
  // Builds the tree for `source_len` choices with branch width <= max_branch_len (2..20), then
  // draws the shuffled (key, choice index) listing.  All randomness comes from `seed`.
  KeyTree(int source_len, int max_branch_len, uint64_t seed);

  // (key, choice index) in the shuffled order presented to the voter, e.g. ("`C``Q`", 7)
  const std::vector<std::pair<std::string, int>>& keys() const { return keys_; }
  int depth() const;  // depth along the first child chain (reference semantics)
  int source_len() const { return source_len_; }
  // Regex alternations "(`A`)|(`B`)..." and "(A)|(B)..." (reference regex_patterns)
  std::pair<std::string, std::string> regex_patterns() const;

  // Vote over the `source_len` choices from a voter's content (and optional logprobs).
  // `logprobs`: per generated token (token text, top alternatives [(text, logprob or NaN)]).
  // Returns nullopt when no key is found (reference: Error::InvalidContent).
  std::optional<std::vector<double>> vote(
      const std::string& content,
      const std::vector<std::pair<std::string, std::vector<std::pair<std::string, double>>>>* logprobs) const;

  // Last non-overlapping, leftmost-first match of any key (with ticks first, then bare);
  // returns the matched key text or empty.
  std::string find_key(const std::string& content) const;

 private:
  std::unique_ptr<KeyNode> build(std::mt19937_64& rng, const std::vector<int>& src, bool force);
  void collect(const KeyNode* n, const std::string& prefix, std::vector<std::pair<std::string, int>>& out) const;

  int source_len_, max_branch_;
  std::unique_ptr<KeyNode> root_;
  std::vector<std::pair<std::string, int>> keys_;
};

// Weighted tally (reference client.rs:384-455) for one request.
//   votes[l] (empty = voter without a vote), weights[l]
// returns (choice_weight[C], confidence[C], voter_confidence[l] (NaN where no vote))
struct TallyResult {
  std::vector<double> choice_weight, confidence, voter_confidence;
};
TallyResult tally(const std::vector<std::vector<double>>& votes, const std::vector<double>& weights, int C);

// Error-code unification when every voter failed (reference client.rs:385-409): same code, else
// 400 if all codes are 4xx, else 500.  `codes` empty => no error.
std::optional<int> unify_error_codes(const std::vector<int>& codes);

}  // namespace lwc
