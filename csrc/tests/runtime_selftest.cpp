// Host-runtime self test built with -fsanitize=address,undefined (sanitizers on host code;
// GPU sanitizers are not available on this pool).  Exercises the paths the engine drives every step:
// block allocation / fork / copy-on-write / free churn, the key tree for many choice counts, vote
// extraction with and without logprobs, tally and error unification.  Exit code 0 = pass; ASan/UBSan
// abort on any memory or UB error.  Driven by tests/test_native_sanitizers.py.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../runtime/block_manager.h"
#include "../runtime/consensus_core.h"

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

static void block_manager_churn() {
  lwc::BlockManager bm(512, 16);
  std::mt19937 rng(7);
  std::vector<int64_t> live;
  int64_t next = 1;
  for (int it = 0; it < 20000; ++it) {
    const int op = rng() % 4;
    if (op == 0 && bm.can_allocate(8)) {
      bm.add_sequence(next, 1 + rng() % 100);
      live.push_back(next++);
    } else if (op == 1 && !live.empty() && bm.num_free() > 4) {
      const int64_t p = live[rng() % live.size()];
      bm.fork(p, next);
      live.push_back(next++);
    } else if (op == 2 && !live.empty()) {
      const int64_t s = live[rng() % live.size()];
      if (bm.num_free() >= bm.append_cost(s)) {
        const int64_t slot = bm.append_token(s);
        CHECK(slot >= 0 && slot < 512 * 16);
        CHECK(bm.slot(s, bm.length(s) - 1) == slot);
      }
    } else if (op == 3 && !live.empty()) {
      const size_t i = rng() % live.size();
      bm.free_sequence(live[i]);
      live.erase(live.begin() + i);
    }
    for (auto& cp : bm.take_copies()) CHECK(cp.first != cp.second);
  }
  for (int64_t s : live) bm.free_sequence(s);
  CHECK(bm.num_free() == 512);
  CHECK(bm.num_sequences() == 0);
}

// prefix cache: prompts drawn from a few shared stems so blocks are reused, resurrected from the LRU
// list and evicted under pressure; every reused block must hold the same tokens as the new prompt
static void prefix_cache_churn() {
  lwc::BlockManager bm(256, 16);
  bm.set_prefix_caching(true);
  std::mt19937 rng(11);
  std::vector<std::vector<int32_t>> stems(6);
  for (auto& st : stems)
    for (int i = 0; i < 80; ++i) st.push_back((int32_t)(rng() % 1000));
  std::vector<std::pair<int64_t, std::vector<int32_t>>> live;
  int64_t next = 1;
  for (int it = 0; it < 5000; ++it) {
    if (rng() % 3 != 0 || live.empty()) {
      std::vector<int32_t> p = stems[rng() % stems.size()];
      p.resize(1 + rng() % p.size());
      for (int i = (int)(rng() % 20); i > 0; --i) p.push_back((int32_t)(rng() % 1000));
      const int need = bm.blocks_for((int64_t)p.size());
      if (!bm.can_allocate(need)) {
        const size_t i = rng() % live.size();
        bm.free_sequence(live[i].first);
        live.erase(live.begin() + i);
        continue;
      }
      const int64_t c = bm.add_sequence_cached(next, p);
      CHECK(c % 16 == 0 && c < (int64_t)p.size());
      const auto& tab = bm.block_table(next);
      for (auto& lv : live)  // a shared block means a shared token prefix up to that block
        for (int64_t b = 0; b < c / 16 && b < (int64_t)bm.block_table(lv.first).size(); ++b)
          if (bm.block_table(lv.first)[b] == tab[b])
            CHECK(std::equal(p.begin(), p.begin() + (b + 1) * 16, lv.second.begin()));
      bm.cache_prefix(next, p);
      live.emplace_back(next++, p);
    } else {
      const size_t i = rng() % live.size();
      bm.free_sequence(live[i].first);
      live.erase(live.begin() + i);
    }
  }
  for (auto& lv : live) bm.free_sequence(lv.first);
  CHECK(bm.num_free() == 256);
  CHECK(bm.num_evictable() == bm.num_cached_blocks());
}

static void key_tree_and_votes() {
  for (int n : {2, 3, 7, 20, 21, 57, 400, 401}) {
    for (int m : {2, 5, 20}) {
      lwc::KeyTree t(n, m, 1234 + n * 31 + m);
      CHECK((int)t.keys().size() == n);
      std::vector<int> seen(n, 0);
      for (auto& kv : t.keys()) seen[kv.second]++;
      for (int c : seen) CHECK(c == 1);
      // every key votes one-hot for its own choice
      for (auto& kv : t.keys()) {
        auto v = t.vote("I pick " + kv.first + " for sure", nullptr);
        CHECK(v.has_value() && (int)v->size() == n);
        CHECK(std::fabs((*v)[kv.second] - 1.0) < 1e-12);
      }
      CHECK(!t.vote("no key here", nullptr).has_value());
    }
  }
  // logprob-weighted vote on a single-level tree
  lwc::KeyTree t(3, 20, 99);
  const std::string key = t.keys()[0].first;  // e.g. "`K`"
  const char letter = key[1];
  std::vector<std::pair<std::string, std::vector<std::pair<std::string, double>>>> lps;
  lps.push_back({"`", {{"`", -0.01}}});
  std::vector<std::pair<std::string, double>> alts = {{std::string(1, letter), std::log(0.6)}};
  for (auto& kv : t.keys())
    if (kv.first != key) alts.push_back({std::string(1, kv.first[1]), std::log(0.2)});
  alts.push_back({"zz", std::log(0.05)});
  alts.push_back({"nan", NAN});
  lps.push_back({std::string(1, letter), alts});
  lps.push_back({"`", {{"`", -0.01}}});
  auto v = t.vote(key, &lps);
  CHECK(v.has_value());
  double sum = 0;
  for (double x : *v) sum += x;
  CHECK(std::fabs(sum - 1.0) < 1e-9);
  CHECK((*v)[t.keys()[0].second] > 0.5);
}

static void tally_and_codes() {
  auto r = lwc::tally({{1, 0, 0}, {}, {0.5, 0.5, 0}}, {1.0, 5.0, 2.0}, 3);
  CHECK(std::fabs(r.choice_weight[0] - 2.0) < 1e-12 && std::fabs(r.choice_weight[1] - 1.0) < 1e-12);
  CHECK(std::fabs(r.confidence[0] + r.confidence[1] + r.confidence[2] - 1.0) < 1e-12);
  CHECK(std::isnan(r.voter_confidence[1]));
  CHECK(lwc::unify_error_codes({404, 404}).value() == 404);
  CHECK(lwc::unify_error_codes({400, 429}).value() == 400);
  CHECK(lwc::unify_error_codes({400, 503}).value() == 500);
  CHECK(!lwc::unify_error_codes({}).has_value());
}

int main() {
  block_manager_churn();
  prefix_cache_churn();
  key_tree_and_votes();
  tally_and_codes();
  std::puts("runtime selftest ok");
  return 0;
}
