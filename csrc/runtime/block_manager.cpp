#include "block_manager.h"

#include <algorithm>
#include <string>

namespace lwc {

BlockManager::BlockManager(int num_blocks, int block_size) : num_blocks_(num_blocks), block_size_(block_size) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("BlockManager: sizes must be positive");
  free_.reserve(num_blocks);
  // pop_back() hands out low block ids first
  for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  ref_.assign(num_blocks, 0);
}

const BlockManager::Seq& BlockManager::get(int64_t seq) const {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) throw std::out_of_range("BlockManager: unknown sequence " + std::to_string(seq));
  return it->second;
}
BlockManager::Seq& BlockManager::get(int64_t seq) {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) throw std::out_of_range("BlockManager: unknown sequence " + std::to_string(seq));
  return it->second;
}

int32_t BlockManager::alloc_block() {
  int32_t b;
  if (!free_.empty()) {
    b = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {  // reclaim the least recently used cached block
    b = lru_.front();
    lru_.pop_front();
    unregister(b);
  } else {
    throw std::runtime_error("BlockManager: out of KV blocks");
  }
  ref_[b] = 1;
  return b;
}

void BlockManager::release(int32_t block) {
  if (ref_[block] <= 0) throw std::logic_error("BlockManager: double free of block " + std::to_string(block));
  if (--ref_[block] == 0) {
    if (registered_.size() && registered_[block])
      lru_pos_[block] = lru_.insert(lru_.end(), block);  // stays resident until the pool needs it
    else
      free_.push_back(block);
  }
}

void BlockManager::acquire_cached(int32_t block) {
  if (ref_[block] == 0) lru_.erase(lru_pos_[block]);
  ++ref_[block];
}

void BlockManager::unregister(int32_t block) {
  if (!registered_[block]) return;
  auto it = by_key_.find(key_[block]);
  if (it != by_key_.end() && it->second == block) by_key_.erase(it);
  registered_[block] = 0;
}

static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

static constexpr uint64_t kRootKey = 0x243f6a8885a308d3ULL;

uint64_t BlockManager::chain_key(uint64_t parent, const int32_t* toks) const {
  uint64_t h = mix64(parent ^ 0x6a09e667f3bcc909ULL);
  for (int i = 0; i < block_size_; ++i) h = mix64(h ^ ((uint64_t)(uint32_t)toks[i] << 1 | 1ULL) ^ (uint64_t)i << 40);
  return h;
}

void BlockManager::set_prefix_caching(bool on) {
  if (on && registered_.empty()) {
    key_.assign(num_blocks_, 0);
    parent_key_.assign(num_blocks_, 0);
    registered_.assign(num_blocks_, 0);
    block_tokens_.assign((size_t)num_blocks_ * block_size_, 0);
    lru_pos_.resize(num_blocks_);
  }
  if (!on) {  // drop the cache: unreferenced cached blocks go back to the free list
    for (int32_t b : lru_) free_.push_back(b);
    lru_.clear();
    by_key_.clear();
    std::fill(registered_.begin(), registered_.end(), 0);
  }
  prefix_caching_ = on;
}

std::vector<int32_t> BlockManager::match_blocks(const std::vector<int32_t>& tokens, int64_t max_blocks) const {
  std::vector<int32_t> out;
  if (!prefix_caching_) return out;
  uint64_t parent = kRootKey;
  for (int64_t i = 0; i < max_blocks; ++i) {
    const int32_t* t = tokens.data() + i * block_size_;
    const uint64_t k = chain_key(parent, t);
    auto it = by_key_.find(k);
    if (it == by_key_.end()) break;
    const int32_t b = it->second;
    if (parent_key_[b] != parent ||
        !std::equal(t, t + block_size_, block_tokens_.begin() + (size_t)b * block_size_))
      break;  // hash collision: treat as a miss
    out.push_back(b);
    parent = k;
  }
  return out;
}

int64_t BlockManager::match_prefix(const std::vector<int32_t>& tokens) const {
  if (tokens.empty()) return 0;
  return (int64_t)match_blocks(tokens, ((int64_t)tokens.size() - 1) / block_size_).size() * block_size_;
}

int64_t BlockManager::add_sequence_cached(int64_t seq, const std::vector<int32_t>& tokens) {
  if (seqs_.count(seq)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(seq));
  const int64_t n = (int64_t)tokens.size();
  const std::vector<int32_t> hit = match_blocks(tokens, n > 0 ? (n - 1) / block_size_ : 0);
  const int need = blocks_for(n) - (int)hit.size();
  // the matched blocks may sit in the LRU list: taking them must not count them as allocatable
  int in_lru = 0;
  for (int32_t b : hit) in_lru += ref_[b] == 0;
  if (num_free() - in_lru < need) throw std::runtime_error("BlockManager: out of KV blocks");
  Seq s;
  s.blocks.reserve(blocks_for(n) + 8);
  for (int32_t b : hit) {
    acquire_cached(b);
    s.blocks.push_back(b);
  }
  for (int i = 0; i < need; ++i) s.blocks.push_back(alloc_block());
  s.len = n;
  seqs_.emplace(seq, std::move(s));
  return (int64_t)hit.size() * block_size_;
}

void BlockManager::cache_prefix(int64_t seq, const std::vector<int32_t>& tokens) {
  if (!prefix_caching_) return;
  const Seq& s = get(seq);
  const int64_t full = std::min<int64_t>((int64_t)tokens.size(), s.len) / block_size_;
  uint64_t parent = kRootKey;
  for (int64_t i = 0; i < full && i < (int64_t)s.blocks.size(); ++i) {
    const int32_t b = s.blocks[i];
    const int32_t* t = tokens.data() + i * block_size_;
    const uint64_t k = chain_key(parent, t);
    if (!registered_[b]) {
      auto it = by_key_.find(k);
      if (it == by_key_.end()) {  // first copy of this prefix block: register it
        registered_[b] = 1;
        key_[b] = k;
        parent_key_[b] = parent;
        std::copy(t, t + block_size_, block_tokens_.begin() + (size_t)b * block_size_);
        by_key_.emplace(k, b);
      }
    }
    parent = k;
  }
}

void BlockManager::add_sequence(int64_t seq, int64_t num_tokens) {
  if (seqs_.count(seq)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(seq));
  const int need = blocks_for(num_tokens);
  if (!can_allocate(need)) throw std::runtime_error("BlockManager: out of KV blocks");
  Seq s;
  s.blocks.reserve(need + 8);
  for (int i = 0; i < need; ++i) s.blocks.push_back(alloc_block());
  s.len = num_tokens;
  seqs_.emplace(seq, std::move(s));
}

void BlockManager::fork(int64_t parent, int64_t child) {
  if (seqs_.count(child)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(child));
  const Seq& p = get(parent);
  Seq c;
  c.blocks = p.blocks;
  c.len = p.len;
  for (int32_t b : c.blocks) ++ref_[b];
  seqs_.emplace(child, std::move(c));
}

int BlockManager::append_cost(int64_t seq) const {
  const Seq& s = get(seq);
  if (s.len % block_size_ == 0) return 1;          // needs a fresh block
  return ref_[s.blocks.back()] > 1 ? 1 : 0;         // copy-on-write of a shared partial block
}

int64_t BlockManager::append_token(int64_t seq) {
  Seq& s = get(seq);
  const int64_t pos = s.len;
  if (pos % block_size_ == 0) {
    s.blocks.push_back(alloc_block());
  } else {
    int32_t& last = s.blocks.back();
    if (ref_[last] > 1) {  // copy-on-write
      const int32_t nb = alloc_block();
      copies_.emplace_back(last, nb);
      --ref_[last];
      last = nb;
    }
  }
  s.len = pos + 1;
  return (int64_t)s.blocks[pos / block_size_] * block_size_ + pos % block_size_;
}

int64_t BlockManager::slot(int64_t seq, int64_t pos) const {
  const Seq& s = get(seq);
  if (pos < 0 || pos >= s.len) throw std::out_of_range("BlockManager: position out of range");
  return (int64_t)s.blocks[pos / block_size_] * block_size_ + pos % block_size_;
}

void BlockManager::free_sequence(int64_t seq) {
  auto it = seqs_.find(seq);
  if (it == seqs_.end()) return;
  for (int32_t b : it->second.blocks) release(b);
  seqs_.erase(it);
}

int64_t BlockManager::append_cost_total(const std::vector<int64_t>& seqs) const {
  int64_t n = 0;
  for (int64_t q : seqs) n += append_cost(q);
  return n;
}

BlockManager::Swapped BlockManager::swap_out(const std::vector<int64_t>& seqs) {
  Swapped out;
  std::unordered_map<int32_t, int32_t> index;
  for (int64_t q : seqs) {
    const Seq& s = get(q);
    std::vector<int32_t> t;
    t.reserve(s.blocks.size());
    for (int32_t b : s.blocks) {
      auto it = index.find(b);
      if (it == index.end()) {
        it = index.emplace(b, (int32_t)out.blocks.size()).first;
        out.blocks.push_back(b);
      }
      t.push_back(it->second);
    }
    out.tables.push_back(std::move(t));
    out.lens.push_back(s.len);
  }
  for (int64_t q : seqs) free_sequence(q);
  return out;
}

std::vector<int32_t> BlockManager::swap_in(const std::vector<int64_t>& seqs, int n,
                                           const std::vector<std::vector<int32_t>>& tables,
                                           const std::vector<int64_t>& lens) {
  if (seqs.size() != tables.size() || seqs.size() != lens.size())
    throw std::invalid_argument("BlockManager::swap_in: seqs / tables / lens size mismatch");
  for (int64_t q : seqs)
    if (seqs_.count(q)) throw std::invalid_argument("BlockManager: sequence exists " + std::to_string(q));
  for (size_t i = 0; i < tables.size(); ++i) {
    if ((int64_t)tables[i].size() != blocks_for(lens[i]))
      throw std::invalid_argument("BlockManager::swap_in: table does not match the length");
    for (int32_t x : tables[i])
      if (x < 0 || x >= n) throw std::out_of_range("BlockManager::swap_in: block index out of range");
  }
  if (!can_allocate(n)) throw std::runtime_error("BlockManager: out of KV blocks");
  std::vector<int32_t> phys(n);
  for (int i = 0; i < n; ++i) phys[i] = alloc_block();  // refcount 1 each
  std::vector<int32_t> refs(n, 0);
  for (const auto& t : tables)
    for (int32_t x : t) ++refs[x];
  for (int i = 0; i < n; ++i) {
    if (refs[i] == 0) {  // exported but referenced by nobody: give it back
      release(phys[i]);
      continue;
    }
    ref_[phys[i]] = refs[i];
  }
  for (size_t i = 0; i < seqs.size(); ++i) {
    Seq s;
    s.blocks.reserve(tables[i].size() + 8);
    for (int32_t x : tables[i]) s.blocks.push_back(phys[x]);
    s.len = lens[i];
    seqs_.emplace(seqs[i], std::move(s));
  }
  return phys;
}

std::vector<std::pair<int32_t, int32_t>> BlockManager::take_copies() {
  std::vector<std::pair<int32_t, int32_t>> out;
  out.swap(copies_);
  return out;
}

}  // namespace lwc
